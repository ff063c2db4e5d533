"""Every `file.rs:N[-M]` citation of the reference in the product, the oracle, the header and the
Rust crates lies inside the cited file (ten citations pointed past the end of their
file).  A citation names a path suffix (`cpu/air.rs`, `crates/stark/src/prover.rs`); it must
resolve to at least one reference file, and every cited line must exist in one of them.  Paths
that resolve to nothing are un-vendored Plonky3 files ([p3-recalled]) and are listed, not
checked.  Needs the reference checkout (this container); skipped where it is absent."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SCANNED = ["zkvm-brainfuck_amd/csrc", "zkvm-brainfuck_amd/bfz", "oracle", "include", "crates"]
EXTS = (".h", ".hip", ".cpp", ".c", ".py", ".rs", ".inc", ".patch")
CITE = re.compile(r"([A-Za-z0-9_./-]*[A-Za-z0-9_]+\.rs):(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)")


def _reference_files():
    out = {}
    for d, dirs, fs in os.walk(REF):
        dirs[:] = [x for x in dirs if x not in (".git", "target")]
        for f in fs:
            if f.endswith(".rs"):
                p = os.path.join(d, f)
                with open(p, errors="replace") as fh:
                    out[os.path.relpath(p, REF)] = sum(1 for _ in fh)
    return out


def _citations():
    for top in SCANNED:
        for d, _, fs in os.walk(os.path.join(ROOT, top)):
            for f in fs:
                if not f.endswith(EXTS):
                    continue
                p = os.path.join(d, f)
                with open(p, errors="replace") as fh:
                    for i, line in enumerate(fh, 1):
                        for m in CITE.finditer(line):
                            yield os.path.relpath(p, ROOT), i, m.group(1), m.group(2)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_reference_citations_are_in_range():
    files = _reference_files()
    bad, checked, unresolved = [], 0, set()
    for src, line, path, spans in _citations():
        path = path.replace(REF + "/", "").replace(REF[1:] + "/", "").lstrip("./")
        cands = [f for f in files if f == path or f.endswith("/" + path)]
        if not cands:
            unresolved.add(path)
            continue
        longest = max(files[c] for c in cands)
        for span in spans.split(","):
            lo, _, hi = span.partition("-")
            lo, hi = int(lo), int(hi or lo)
            checked += 1
            if not (1 <= lo <= hi <= longest):
                bad.append(f"{src}:{line}: {path}:{span} (file has {longest} lines)")
    assert checked > 300, checked  # the scan found the citations
    assert not bad, "\n".join(bad)


def test_profiler_ranges_use_the_reference_span_names():
    """The roctx ranges of prover.hip (gpu.h Span) carry the names of the reference's tracing
    spans (crates/stark/src/prover.rs), so a rocprofv3 --marker-trace of bfz lines up with a
    tracing log of the reference; a range without a reference span says so in its comment."""
    ref = os.path.join(REF, "crates/stark/src/prover.rs")
    if not os.path.exists(ref):
        pytest.skip("reference checkout absent")
    spans = set(re.findall(r'_span!\((?:parent: &\w+, )?"([^"]+)"', open(ref).read()))
    src = open(os.path.join(ROOT, "zkvm-brainfuck_amd/csrc/prover.hip")).read()
    names = re.findall(r'(?:Span \w+\(|span\.begin\()"([^"]+)"\);(.*)', src)
    assert len(names) >= 7
    for name, comment in names:
        assert name in spans or "no span of its own in the reference" in comment, name
