"""Independent Python model of the two proof byte forms -- TEST INFRASTRUCTURE.

Parses the BFZ1 normal form into plain Python values and re-emits it either as BFZ1 or as
bincode::serialize(&ShardProof<KoalaBearPoseidon2>) (crates/stark/src/types.rs:66-73; bincode
1.x defaults: little-endian fixed-width ints, u64 lengths for Vec/String/HashMap, structs and
fixed arrays without length).  Written separately from csrc/proof.cpp so the C++ encoder is
checked against a second implementation, and used to build tampered proofs.
"""
import struct

P = 0x7F000001
R = (1 << 32) % P
CHIPS = ("Cpu", "Program", "AddSub", "Jump", "Memory", "Byte", "MemoryInstrs", "IO")


class _R:
    def __init__(self, b):
        self.b, self.o = b, 0

    def u32(self):
        v = struct.unpack_from("<I", self.b, self.o)[0]
        self.o += 4
        return v

    def words(self, k):
        v = list(struct.unpack_from("<%dI" % k, self.b, self.o))
        self.o += 4 * k
        return v


def parse_bfz1(b: bytes) -> dict:
    """Canonical field values throughout."""
    r = _R(b)
    assert r.u32() == 0x315A4642
    nc = r.u32()
    chips = []
    for _ in range(nc):
        cid = r.u32()
        ln = r.u32()
        name = b[r.o:r.o + ln].decode()
        r.o += ln
        assert name == CHIPS[cid]
        chips.append(cid)
    pf = {"chips": chips, "roots": [r.words(8) for _ in range(3)], "opened": []}

    def efs():
        k = r.u32()
        return [r.words(4) for _ in range(k)]

    for _ in range(nc):
        o = {"log_degree": r.u32()}
        for key in ("prep_local", "prep_next", "main_local", "main_next", "perm_local",
                    "perm_next"):
            o[key] = efs()
        assert r.u32() == 2
        o["quotient"] = [efs(), efs()]
        o["cumsum"] = r.words(4)
        pf["opened"].append(o)
    pf["commit_roots"] = [r.words(8) for _ in range(r.u32())]
    queries = []
    for _ in range(r.u32()):
        inputs = []
        for _ in range(r.u32()):
            rows = [r.words(r.u32()) for _ in range(r.u32())]
            path = [r.words(8) for _ in range(r.u32())]
            inputs.append({"rows": rows, "path": path})
        steps = []
        for _ in range(r.u32()):
            sib = r.words(4)
            steps.append({"sibling": sib, "path": [r.words(8) for _ in range(r.u32())]})
        queries.append({"inputs": inputs, "steps": steps})
    pf["queries"] = queries
    pf["final_poly"] = r.words(4)
    pf["pow_witness"] = r.u32()
    assert r.o == len(b)
    return pf


class _W:
    def __init__(self, mont: bool, u64len: bool):
        self.parts, self.mont, self.u64len = [], mont, u64len

    def u32(self, v):
        self.parts.append(struct.pack("<I", v))

    def u64(self, v):
        self.parts.append(struct.pack("<Q", v))

    def len(self, k):
        self.u64(k) if self.u64len else self.u32(k)

    def fps(self, vals):
        if self.mont:
            vals = [(v * R) % P for v in vals]
        self.parts.append(struct.pack("<%dI" % len(vals), *vals))

    def efs(self, v):
        self.len(len(v))
        for e in v:
            self.fps(e)

    def digests(self, v):
        self.len(len(v))
        for d in v:
            self.fps(d)

    def bytes(self):
        return b"".join(self.parts)


def encode_bfz1(pf: dict) -> bytes:
    w = _W(False, False)
    w.u32(0x315A4642)
    w.u32(len(pf["chips"]))
    for c in pf["chips"]:
        w.u32(c)
        w.u32(len(CHIPS[c]))
        w.parts.append(CHIPS[c].encode())
    for d in pf["roots"]:
        w.fps(d)
    for o in pf["opened"]:
        w.u32(o["log_degree"])
        for key in ("prep_local", "prep_next", "main_local", "main_next", "perm_local",
                    "perm_next"):
            w.efs(o[key])
        w.u32(2)
        w.efs(o["quotient"][0])
        w.efs(o["quotient"][1])
        w.fps(o["cumsum"])
    _fri(w, pf)
    return w.bytes()


def _fri(w, pf):
    w.digests(pf["commit_roots"])
    w.len(len(pf["queries"]))
    for q in pf["queries"]:
        w.len(len(q["inputs"]))
        for b in q["inputs"]:
            w.len(len(b["rows"]))
            for row in b["rows"]:
                w.len(len(row))
                w.fps(row)
            w.digests(b["path"])
        w.len(len(q["steps"]))
        for s in q["steps"]:
            w.fps(s["sibling"])
            w.digests(s["path"])
    w.fps(pf["final_poly"])
    w.fps([pf["pow_witness"]])


def encode_bincode(pf: dict, montgomery: bool = True) -> bytes:
    w = _W(montgomery, True)
    for d in pf["roots"]:                      # ShardCommitment (3 x Hash<Val, Val, 8>)
        w.fps(d)
    w.len(len(pf["opened"]))                   # ShardOpenedValues.chips
    for o in pf["opened"]:
        for key in ("prep_local", "prep_next", "main_local", "main_next", "perm_local",
                    "perm_next"):
            w.efs(o[key])
        w.len(2)
        w.efs(o["quotient"][0])
        w.efs(o["quotient"][1])
        w.fps(o["cumsum"])
        w.u64(o["log_degree"])
    _fri(w, pf)                                # FriProof
    w.len(len(pf["chips"]))                    # chip_ordering, proof order
    for i, c in enumerate(pf["chips"]):
        w.len(len(CHIPS[c]))
        w.parts.append(CHIPS[c].encode())
        w.u64(i)
    return w.bytes()


class _B:
    """bincode reader (u64 lengths); field words converted out of Montgomery form if asked."""

    def __init__(self, b, mont: bool):
        self.b, self.o, self.mont = b, 0, mont
        self.rinv = pow(R, -1, P)

    def u32(self):
        v = struct.unpack_from("<I", self.b, self.o)[0]
        self.o += 4
        return v

    def u64(self):
        v = struct.unpack_from("<Q", self.b, self.o)[0]
        self.o += 8
        return v

    def fps(self, k):
        v = list(struct.unpack_from("<%dI" % k, self.b, self.o))
        self.o += 4 * k
        if any(x >= P for x in v):
            raise ValueError("field word out of range")
        return [(x * self.rinv) % P for x in v] if self.mont else v

    def efs(self):
        return [self.fps(4) for _ in range(self.u64())]

    def digests(self):
        return [self.fps(8) for _ in range(self.u64())]


def decode_bincode(b: bytes, montgomery: bool = True) -> dict:
    """Inverse of encode_bincode: the same dict parse_bfz1 returns (canonical values).  The
    chip_ordering map may come in any order (a Rust HashMap); chips are put in index order."""
    r = _B(b, montgomery)
    pf = {"roots": [r.fps(8) for _ in range(3)], "opened": []}
    for _ in range(r.u64()):
        o = {}
        for key in ("prep_local", "prep_next", "main_local", "main_next", "perm_local",
                    "perm_next"):
            o[key] = r.efs()
        if r.u64() != 2:
            raise ValueError("quotient chunk count")
        o["quotient"] = [r.efs(), r.efs()]
        o["cumsum"] = r.fps(4)
        o["log_degree"] = r.u64()
        pf["opened"].append(o)
    pf["commit_roots"] = r.digests()
    queries = []
    for _ in range(r.u64()):
        inputs = []
        for _ in range(r.u64()):
            rows = [r.fps(r.u64()) for _ in range(r.u64())]
            inputs.append({"rows": rows, "path": r.digests()})
        steps = []
        for _ in range(r.u64()):
            sib = r.fps(4)
            steps.append({"sibling": sib, "path": r.digests()})
        queries.append({"inputs": inputs, "steps": steps})
    pf["queries"] = queries
    pf["final_poly"] = r.fps(4)
    pf["pow_witness"] = r.fps(1)[0]
    # chip_ordering: HashMap<String, usize>, written as (len, name bytes, u64 index) pairs
    n = r.u64()
    n_opened = len(pf["opened"])
    order = {}
    for _ in range(n):
        ln = r.u64()
        name = r.b[r.o:r.o + ln].decode()
        r.o += ln
        order[r.u64()] = CHIPS.index(name)
    if r.o != len(r.b) or sorted(order) != list(range(n)) or n != n_opened:
        raise ValueError("trailing bytes or malformed chip ordering")
    pf["chips"] = [order[i] for i in range(n)]
    return pf
