// ShardProof byte forms (see proof.h).  Decoders bound every length by the bytes that remain,
// so malformed input throws instead of allocating.
#include "proof.h"

#include <cstring>
#include <stdexcept>
#include <string>

#include "machine.h"

namespace bfz {

using namespace kb;

namespace {

constexpr uint32_t BFZ1_MAGIC = 0x315a4642u;

struct Out {
  std::vector<uint8_t> b;
  FieldRepr repr = FieldRepr::CANONICAL;
  bool u64len = false;  // bincode: u64 lengths; BFZ1: u32
  void put(const void* p, size_t n) {
    const uint8_t* q = static_cast<const uint8_t*>(p);
    b.insert(b.end(), q, q + n);
  }
  void u32(uint32_t v) { put(&v, 4); }
  void u64(uint64_t v) { put(&v, 8); }
  void len(size_t n) {
    if (u64len) u64(n);
    else u32((uint32_t)n);
  }
  void fp(uint32_t mont) { u32(repr == FieldRepr::MONTGOMERY ? mont : from_mont(mont)); }
  void ef(const EF& e) {
    for (int i = 0; i < 4; i++) fp(e.c[i]);
  }
  void digest(const Digest& d) {
    for (uint32_t x : d) fp(x);
  }
  void efs(const std::vector<EF>& v) {
    len(v.size());
    for (const EF& e : v) ef(e);
  }
  void digests(const std::vector<Digest>& v) {
    len(v.size());
    for (const Digest& d : v) digest(d);
  }
  void words(const std::vector<uint32_t>& v) {
    len(v.size());
    for (uint32_t x : v) fp(x);
  }
};

struct In {
  const uint8_t* p;
  size_t n, off = 0;
  FieldRepr repr = FieldRepr::CANONICAL;
  bool u64len = false;
  void need(size_t k) {
    if (k > n - off) throw std::runtime_error("truncated proof");
  }
  uint32_t u32() {
    need(4);
    uint32_t v;
    std::memcpy(&v, p + off, 4);
    off += 4;
    return v;
  }
  uint64_t u64() {
    need(8);
    uint64_t v;
    std::memcpy(&v, p + off, 8);
    off += 8;
    return v;
  }
  // a length whose elements take at least `min_elem` bytes each
  size_t len(size_t min_elem) {
    const uint64_t k = u64len ? u64() : u32();
    if (min_elem && k > (n - off) / min_elem) throw std::runtime_error("bad length in proof");
    return (size_t)k;
  }
  uint32_t fp() {
    const uint32_t v = u32();
    if (v >= P) throw std::runtime_error("non-canonical field element");
    return repr == FieldRepr::MONTGOMERY ? v : to_mont(v);
  }
  EF ef() {
    EF e;
    for (int i = 0; i < 4; i++) e.c[i] = fp();
    return e;
  }
  Digest digest() {
    Digest d;
    for (auto& x : d) x = fp();
    return d;
  }
  std::vector<EF> efs() {
    std::vector<EF> v(len(16));
    for (EF& e : v) e = ef();
    return v;
  }
  std::vector<Digest> digests() {
    std::vector<Digest> v(len(32));
    for (Digest& d : v) d = digest();
    return v;
  }
  std::vector<uint32_t> words() {
    std::vector<uint32_t> v(len(4));
    for (uint32_t& x : v) x = fp();
    return v;
  }
};

int chip_by_name(const std::string& s) {
  for (int c = 0; c < NUM_CHIPS; c++)
    if (s == CHIP_INFO[c].name) return c;
  throw std::runtime_error("unknown chip name in proof: " + s);
}

}  // namespace

// ------------------------------------------------------------------------------------ BFZ1
ShardProof decode_bfz1(const uint8_t* p, size_t n) {
  In r{p, n};
  ShardProof pf;
  if (r.u32() != BFZ1_MAGIC) throw std::runtime_error("bad magic");
  const uint32_t nc = r.u32();
  if (nc == 0 || nc > NUM_CHIPS) throw std::runtime_error("bad chip count");
  std::vector<bool> seen(NUM_CHIPS, false);
  for (uint32_t i = 0; i < nc; i++) {
    const uint32_t c = r.u32();
    if (c >= (uint32_t)NUM_CHIPS || seen[c]) throw std::runtime_error("bad chip id");
    seen[c] = true;
    const size_t l = r.len(1);
    r.need(l);
    if (l != std::strlen(CHIP_INFO[c].name) || std::memcmp(p + r.off, CHIP_INFO[c].name, l) != 0)
      throw std::runtime_error("chip name mismatch");
    r.off += l;
    pf.chips.push_back((int)c);
  }
  pf.main_root = r.digest();
  pf.perm_root = r.digest();
  pf.quot_root = r.digest();
  pf.opened.resize(nc);
  for (uint32_t i = 0; i < nc; i++) {
    ChipOpened& c = pf.opened[i];
    c.chip = pf.chips[i];
    c.log_degree = r.u32();
    c.prep_local = r.efs();
    c.prep_next = r.efs();
    c.main_local = r.efs();
    c.main_next = r.efs();
    c.perm_local = r.efs();
    c.perm_next = r.efs();
    if (r.u32() != 2) throw std::runtime_error("bad quotient chunk count");
    c.quotient[0] = r.efs();
    c.quotient[1] = r.efs();
    c.cumsum = r.ef();
  }
  pf.commit_roots.resize(r.len(32));
  for (Digest& d : pf.commit_roots) d = r.digest();
  pf.queries.resize(r.len(4));
  for (QueryProof& q : pf.queries) {
    q.inputs.resize(r.len(8));
    for (BatchOpening& b : q.inputs) {
      b.rows.resize(r.len(4));
      for (auto& row : b.rows) row = r.words();
      b.path = r.digests();
    }
    q.steps.resize(r.len(20));
    for (CommitPhaseStep& s : q.steps) {
      s.sibling = r.ef();
      s.path = r.digests();
    }
  }
  pf.final_poly = r.ef();
  pf.pow_witness = r.fp();
  if (r.off != n) throw std::runtime_error("trailing bytes");
  return pf;
}

std::vector<uint8_t> encode_bfz1(const ShardProof& pf) {
  Out w;
  w.u32(BFZ1_MAGIC);
  w.u32((uint32_t)pf.chips.size());
  for (int c : pf.chips) {
    const char* nm = CHIP_INFO[c].name;
    w.u32((uint32_t)c);
    w.u32((uint32_t)std::strlen(nm));
    w.put(nm, std::strlen(nm));
  }
  w.digest(pf.main_root);
  w.digest(pf.perm_root);
  w.digest(pf.quot_root);
  for (const ChipOpened& c : pf.opened) {
    w.u32(c.log_degree);
    w.efs(c.prep_local);
    w.efs(c.prep_next);
    w.efs(c.main_local);
    w.efs(c.main_next);
    w.efs(c.perm_local);
    w.efs(c.perm_next);
    w.u32(2);
    w.efs(c.quotient[0]);
    w.efs(c.quotient[1]);
    w.ef(c.cumsum);
  }
  w.digests(pf.commit_roots);
  w.len(pf.queries.size());
  for (const QueryProof& q : pf.queries) {
    w.len(q.inputs.size());
    for (const BatchOpening& b : q.inputs) {
      w.len(b.rows.size());
      for (const auto& row : b.rows) w.words(row);
      w.digests(b.path);
    }
    w.len(q.steps.size());
    for (const CommitPhaseStep& s : q.steps) {
      w.ef(s.sibling);
      w.digests(s.path);
    }
  }
  w.ef(pf.final_poly);
  w.fp(pf.pow_witness);
  return std::move(w.b);
}

// ---------------------------------------------------------------------------------- bincode
// Field order follows the serde derives: ShardProof { commitment, opened_values, opening_proof,
// chip_ordering } (types.rs:66-73).
std::vector<uint8_t> encode_bincode(const ShardProof& pf, FieldRepr repr) {
  Out w;
  w.repr = repr;
  w.u64len = true;
  // commitment: ShardCommitment { main_commit, permutation_commit, quotient_commit }
  // (types.rs:30-35); a Hash<Val, Val, 8> is a fixed array + PhantomData: 8 words, no length
  w.digest(pf.main_root);
  w.digest(pf.perm_root);
  w.digest(pf.quot_root);
  // opened_values: ShardOpenedValues { chips: Vec<ChipOpenedValues> } (types.rs:54-57)
  w.len(pf.opened.size());
  for (const ChipOpened& c : pf.opened) {
    w.efs(c.prep_local);  // preprocessed: AirOpenedValues { local, next } (types.rs:37-42)
    w.efs(c.prep_next);
    w.efs(c.main_local);
    w.efs(c.main_next);
    w.efs(c.perm_local);
    w.efs(c.perm_next);
    w.len(2);             // quotient: Vec<Vec<Challenge>>
    w.efs(c.quotient[0]);
    w.efs(c.quotient[1]);
    w.ef(c.cumsum);       // cumulative_sum: Challenge = [Val; 4], no length
    w.u64(c.log_degree);  // log_degree: usize
  }
  // opening_proof: FriProof { commit_phase_commits, query_proofs, final_poly, pow_witness }
  w.digests(pf.commit_roots);
  w.len(pf.queries.size());
  for (const QueryProof& q : pf.queries) {
    w.len(q.inputs.size());  // input_proof: Vec<BatchOpening { opened_values, opening_proof }>
    for (const BatchOpening& b : q.inputs) {
      w.len(b.rows.size());
      for (const auto& row : b.rows) w.words(row);
      w.digests(b.path);
    }
    w.len(q.steps.size());   // commit_phase_openings: Vec<CommitPhaseProofStep>
    for (const CommitPhaseStep& s : q.steps) {
      w.ef(s.sibling);
      w.digests(s.path);
    }
  }
  w.ef(pf.final_poly);
  w.fp(pf.pow_witness);
  // chip_ordering: HashMap<String, usize> -- normal form: entries in proof order
  w.len(pf.chips.size());
  for (size_t i = 0; i < pf.chips.size(); i++) {
    const char* nm = CHIP_INFO[pf.chips[i]].name;
    w.len(std::strlen(nm));
    w.put(nm, std::strlen(nm));
    w.u64(i);
  }
  return std::move(w.b);
}

ShardProof decode_bincode(const uint8_t* p, size_t n, FieldRepr repr) {
  In r{p, n};
  r.repr = repr;
  r.u64len = true;
  ShardProof pf;
  pf.main_root = r.digest();
  pf.perm_root = r.digest();
  pf.quot_root = r.digest();
  const size_t nc = r.len(16 * 9 + 8 + 8 * 9);
  if (nc == 0 || nc > NUM_CHIPS) throw std::runtime_error("bad chip count");
  pf.opened.resize(nc);
  for (ChipOpened& c : pf.opened) {
    c.prep_local = r.efs();
    c.prep_next = r.efs();
    c.main_local = r.efs();
    c.main_next = r.efs();
    c.perm_local = r.efs();
    c.perm_next = r.efs();
    if (r.len(8) != 2) throw std::runtime_error("bad quotient chunk count");
    c.quotient[0] = r.efs();
    c.quotient[1] = r.efs();
    c.cumsum = r.ef();
    const uint64_t lg = r.u64();
    if (lg > 64) throw std::runtime_error("log degree out of range");
    c.log_degree = (uint32_t)lg;
  }
  pf.commit_roots = r.digests();
  pf.queries.resize(r.len(16));
  for (QueryProof& q : pf.queries) {
    q.inputs.resize(r.len(16));
    for (BatchOpening& b : q.inputs) {
      b.rows.resize(r.len(8));
      for (auto& row : b.rows) row = r.words();
      b.path = r.digests();
    }
    q.steps.resize(r.len(24));
    for (CommitPhaseStep& s : q.steps) {
      s.sibling = r.ef();
      s.path = r.digests();
    }
  }
  pf.final_poly = r.ef();
  pf.pow_witness = r.fp();
  const size_t ne = r.len(17);
  if (ne != nc) throw std::runtime_error("chip_ordering size differs from the opened chips");
  pf.chips.assign(nc, -1);
  std::vector<bool> seen(NUM_CHIPS, false);
  for (size_t k = 0; k < ne; k++) {
    const size_t l = r.len(1);
    r.need(l);
    const std::string name(reinterpret_cast<const char*>(p + r.off), l);
    r.off += l;
    const uint64_t idx = r.u64();
    const int c = chip_by_name(name);
    if (idx >= nc || pf.chips[idx] != -1 || seen[c])
      throw std::runtime_error("chip_ordering is not a bijection onto the opened chips");
    seen[c] = true;
    pf.chips[idx] = c;
  }
  for (size_t i = 0; i < nc; i++) pf.opened[i].chip = pf.chips[i];
  if (r.off != n) throw std::runtime_error("trailing bytes");
  return pf;
}

}  // namespace bfz
