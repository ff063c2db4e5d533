"""Source hash of libbfz.so (build provenance).

The Makefile compiles this hash into the library (bfz_build_id) and bfz._lib refuses to load
a library whose hash differs from the sources next to it, so a stale libbfz.so can never
stand in for HEAD.  Hashed: every file under csrc/ plus include/bfz.h, sorted by path, each
as "<relative path>\\0<bytes>".  Run as a script it prints the hash (used by the Makefile).
"""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)


def files():
    out = []
    csrc = os.path.join(PKG, "csrc")
    for name in sorted(os.listdir(csrc)):
        p = os.path.join(csrc, name)
        if os.path.isfile(p) and not name.startswith("."):
            out.append(("csrc/" + name, p))
    out.append(("include/bfz.h", os.path.join(ROOT, "include", "bfz.h")))
    return out


def source_hash() -> str:
    h = hashlib.sha256()
    for rel, p in files():
        h.update(rel.encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
