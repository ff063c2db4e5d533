// HIP core prover (host orchestration).  Mirrors, stage for stage:
//   MachineProver::prove          crates/stark/src/prover.rs:560-582 (observe_into :595-601)
//   CpuProver::commit             prover.rs:209-236  (sort by (Reverse(height), name))
//   CpuProver::open               prover.rs:242-553  (LogUp, quotient, PCS open, proof)
//   StarkMachine::setup           crates/stark/src/machine.rs:154-224
// and the p3 TwoAdicFriPcs::{commit, open} / fri::prover [p3-recalled].  All bulk data stays
// in HBM; only digests, challenges, opened values and the query openings cross to the host.
#include "prover.h"
#include "pipeline.h"

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "fri.h"
#include "host_p2.h"
#include "logup.h"
#include "ntt.h"
#include "poseidon2.h"
#include "quotient.h"
#include "tracegen.h"
#include "verifier.h"

namespace bfz {

using namespace kb;

static constexpr int LOG_BLOWUP = 1;
static constexpr int POW_BITS = 16;

// kb31_poseidon2.rs:59-62: `value.parse().unwrap()` into a usize -- anything but a whole
// positive decimal number is an error (the reference panics), never a silent 0 or default.
int num_queries_from_env() {
  const char* s = std::getenv("FRI_QUERIES");
  if (!s) return 84;
  char* end = nullptr;
  errno = 0;
  const long v = std::strtol(s, &end, 10);
  if (errno || end == s || *end != '\0' || v <= 0 || v > 4096)
    throw std::runtime_error(std::string("FRI_QUERIES is not a positive query count: '") + s + "'");
  return (int)v;
}

bool observe_openings_from_env() {
  const char* s = std::getenv("BFZ_OBSERVE_OPENINGS");
  if (!s) return true;
  if (!std::strcmp(s, "1")) return true;
  if (!std::strcmp(s, "0")) return false;
  throw std::runtime_error(std::string("BFZ_OBSERVE_OPENINGS must be 0 or 1, not '") + s + "'");
}

// ------------------------------------------------------------------------ challenger
void Challenger::duplex() {
  for (int i = 0; i < nin; i++) st[i] = in[i];
  nin = 0;
  host_permute(st);
  for (int i = 0; i < 8; i++) out[i] = st[i];
  nout = 8;
}
void Challenger::observe(uint32_t v) {
  nout = 0;
  in[nin++] = v;
  if (nin == 8) duplex();
}
void Challenger::observe_digest(const uint32_t d[8]) {
  for (int i = 0; i < 8; i++) observe(d[i]);
}
void Challenger::observe_ef(const EF& e) {
  for (int i = 0; i < 4; i++) observe(e.c[i]);
}
uint32_t Challenger::sample() {
  if (nin > 0 || nout == 0) duplex();
  return out[--nout];
}
EF Challenger::sample_ef() {
  EF r;
  for (int i = 0; i < 4; i++) r.c[i] = sample();
  return r;
}
uint32_t Challenger::sample_bits(int bits) { return from_mont(sample()) & ((1u << bits) - 1); }
bool Challenger::check_witness(int bits, uint32_t w) {
  observe(to_mont(w));
  return sample_bits(bits) == 0;
}

// ------------------------------------------------------------------------ timing
constexpr int MAX_FRI_ROUNDS = 32;
struct FriTail {
  const uint32_t* root[MAX_FRI_ROUNDS];
  int nroots;
  const uint32_t* state;
  const EF* fin;
};
// packed = [root 0 .. root MAX-1 (8 words each) | state (16) | final layer (2 EF)]; nroots may
// be 0 (state then unused)
__global__ void k_pack_fri_tail(FriTail t, uint32_t* __restrict__ packed) {
  const int i = threadIdx.x;
  if (i < 8 * t.nroots) packed[i] = t.root[i >> 3][i & 7];
  if (i < 16) packed[8 * MAX_FRI_ROUNDS + i] = t.state[i];
  if (i < 8) packed[8 * MAX_FRI_ROUNDS + 16 + i] = t.fin[i >> 2].c[i & 3];
}

namespace {
// BFZ_HOST_TRACE=1: host timestamps (us since the last mark 0) at the transcript points of each
// proof, printed on stderr at exit -- splits the GPU's idle gaps into host work and launch
// latency (scripts/hostgap.py).  The marks are kept in memory: an fprintf per mark cost tens
// of microseconds on the GPU boxes and doubled the idle time it was measuring.
// BFZ_HOST_TRACE=live: each mark is printed at once with its lane (where a stalled proof lane
// stands).
struct HostTrace {
  bool on = std::getenv("BFZ_HOST_TRACE") != nullptr;
  bool live = on && std::string(std::getenv("BFZ_HOST_TRACE")) == "live";
  struct Mark {
    std::chrono::steady_clock::time_point t;
    const char* what;  // string literals only
    bool reset;
  };
  std::vector<Mark> marks;
  std::mutex mu;  // the proof lanes mark concurrently
  HostTrace() {
    if (on) marks.reserve(1 << 16);
  }
  void mark(const char* what, bool reset = false) {
    if (!on) return;
    std::lock_guard<std::mutex> lk(mu);
    if (live) {
      std::fprintf(stderr, "host lane %d: %s\n", lane().id, what);
      std::fflush(stderr);
      return;
    }
    if (marks.size() >= (1u << 20)) return;
    marks.push_back({std::chrono::steady_clock::now(), what, reset});
  }
  ~HostTrace() {
    std::chrono::steady_clock::time_point t0{};
    for (const Mark& m : marks) {
      if (m.reset) t0 = m.t;
      std::fprintf(stderr, "host %9.1f %s (abs %.1f)\n",
                   std::chrono::duration<double, std::micro>(m.t - t0).count(), m.what,
                   std::chrono::duration<double, std::micro>(m.t.time_since_epoch()).count());
    }
  }
};
HostTrace& htrace() {
  static HostTrace h;
  return h;
}
}  // namespace
void host_mark(const char* what) { htrace().mark(what); }

// Proof buffers come back through bfz_free and are reused: a fresh 1 MB vector costs a page fault
// per 4 KB page on first touch (hundreds of microseconds on a busy host).
static std::mutex g_pb_mu;
static std::vector<std::vector<uint8_t>> g_pb;
std::vector<uint8_t> acquire_proof_buffer() {
  std::lock_guard<std::mutex> lk(g_pb_mu);
  if (g_pb.empty()) return {};
  std::vector<uint8_t> v = std::move(g_pb.back());
  g_pb.pop_back();
  return v;
}
void release_proof_buffer(std::vector<uint8_t>&& v) {
  std::lock_guard<std::mutex> lk(g_pb_mu);
  if (g_pb.size() < 4) g_pb.push_back(std::move(v));
}
namespace {
struct EvTimer {
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
  std::vector<double*> dst;
  std::vector<double> bytes;
  hipEvent_t begin(hipStream_t st) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(e, st));
    return e;
  }
  void end(hipEvent_t b, hipStream_t st, double* into) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(e, st));
    evs.push_back({b, e});
    dst.push_back(into);
  }
  void collect() {
    for (size_t i = 0; i < evs.size(); i++) {
      HIP_CHECK(hipEventSynchronize(evs[i].second));
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, evs[i].first, evs[i].second));
      *dst[i] += ms;
      HIP_CHECK(hipEventDestroy(evs[i].first));
      HIP_CHECK(hipEventDestroy(evs[i].second));
    }
    evs.clear();
    dst.clear();
  }
};

// An asynchronous device -> host copy into a pinned buffer, waited for later by spinning on its
// event (fetch() waits at once).  Process-global instances rely on the API lock.
struct Mailbox {
  uint8_t* box = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
  void post(const void* src, size_t bytes, hipStream_t st) {
    if (!ev) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    if (pending) HIP_CHECK(hipEventSynchronize(ev));  // a post never waited for (an error path)
    if (bytes > cap) {
      if (box) HIP_CHECK(hipHostFree(box));
      cap = std::max(bytes, (size_t)4096);
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&box), cap, hipHostMallocDefault));
    }
    HIP_CHECK(hipMemcpyAsync(box, src, bytes, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipEventRecord(ev, st));
    pending = true;
  }
  void reserve(size_t bytes) {  // setup: the pinned box and event before the first proof
    if (!ev) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    if (bytes > cap && !pending) {
      if (box) HIP_CHECK(hipHostFree(box));
      cap = std::max(bytes, (size_t)4096);
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&box), cap, hipHostMallocDefault));
    }
  }
  void wait(void* dst, size_t bytes) {
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) HIP_CHECK(e);
    }
    pending = false;
    std::memcpy(dst, box, bytes);
  }
};

void to_canon_digest(const uint32_t* d, uint32_t* o) {
  for (int i = 0; i < 8; i++) o[i] = from_mont(d[i]);
}

struct Writer {  // appends through a cursor into a buffer sized up front (one fill, no per-word resize)
  std::vector<uint8_t> b;
  size_t n = 0;
  void reserve(size_t cap) {
    b = acquire_proof_buffer();  // a returned proof's pages: no page faults on the ~1 MB
    b.resize(cap);
  }
  uint8_t* room(size_t k) {
    if (n + k > b.size()) b.resize(std::max(2 * b.size(), n + k));
    uint8_t* p = b.data() + n;
    n += k;
    return p;
  }
  void u32(uint32_t v) { std::memcpy(room(4), &v, 4); }
  void fp(uint32_t mont) { u32(from_mont(mont)); }
  void raw(const uint32_t* w, size_t k) { std::memcpy(room(4 * k), w, 4 * k); }  // canonical words
  void ef(const EF& e) {
    uint32_t v[4];
    for (int i = 0; i < 4; i++) v[i] = from_mont(e.c[i]);
    std::memcpy(room(16), v, 16);
  }
  void digest(const uint32_t* d) {
    uint32_t v[8];
    for (int i = 0; i < 8; i++) v[i] = from_mont(d[i]);
    std::memcpy(room(32), v, 32);
  }
  void bytes(const void* p, size_t k) { std::memcpy(room(k), p, k); }
  std::vector<uint8_t> take() {
    b.resize(n);
    return std::move(b);
  }
};}  // namespace

void Round::commit(hipStream_t st, bool fetch_root) {
  std::vector<MatRef> refs;
  for (CMat& m : mats) refs.push_back(m.ref());
  merkle_build(refs, tree, st, fetch_root);
}

namespace {
// How one proof is split over the ranks of a shard context.  Rank k owns the
// bit-reversed positions [k H/G, (k+1) H/G) of every vector of height H >= G * 1024 (LDEs,
// Merkle layers, reduced openings, FRI layers): the natural rows i = r (mod G), r = bitrev_G(k).
// Shorter vectors are replicated.
struct Plan {
  int G = 1, lg = 0, k = 0, r = 0;
  int r2 = 0, k2 = 0;  // residue class of the quotient's next rows (i + 2) and its owner
  bool on() const { return G > 1; }
  bool sharded(size_t H) const { return G > 1 && H >= (size_t)G * SHARD_MIN_LEAVES; }
  size_t blk(size_t H) const { return H >> lg; }
  size_t row0(size_t H) const { return (size_t)k * blk(H); }
};
Plan make_plan() {
  Plan p;
  const ShardCtx* c = shard_ctx();
  if (!c || c->world <= 1) return p;
  p.G = c->world;
  p.lg = log2i((size_t)p.G);
  p.k = c->rank;
  p.r = (int)bitrev32((uint32_t)p.k, p.lg);
  p.r2 = (p.r + 2) % p.G;
  p.k2 = (int)bitrev32((uint32_t)p.r2, p.lg);
  return p;
}
}  // namespace

// Columns each chip reads at the next row (verifier.cpp: next_row_columns), computed once.
static const NextCols& chip_next_cols(int chip) {
  static const auto all = [] {
    std::array<NextCols, NUM_CHIPS> a;
    for (int c = 0; c < NUM_CHIPS; c++) a[c] = next_row_columns(c);
    return a;
  }();
  return all[chip];
}

// plan != nullptr and a height it shards: this rank's residue-class shard of the LDE from the
// interpolant's coefficients (kept in cm.coef), plus -- for G >= 4 -- the shard of the next-row
// residue class for the columns in next_cols (the quotient reads only those at row i + 2).
// split (timed proofs only): where the iDFT and the fold + forward DFT time go (the LogUp
// stage's parts); the unsharded coset LDE counts as forward DFT
struct LdeSplit {
  double* idft;
  double* dft;
};
static void lde_into(CMat& cm, const uint32_t* evals, size_t n, int w, uint32_t domain_shift,
                     hipStream_t st, EvTimer* tm, StageTimes* times, const Plan* plan = nullptr,
                     const std::vector<int>* next_cols = nullptr, const LdeSplit* split = nullptr) {
  const bool timed = split && tm && tm->on;
  for (int c = 0; c < 64; c++) cm.nmap[c] = (uint8_t)c;
  cm.n = n;
  cm.log_n = log2i(n);
  cm.shift = domain_shift;
  cm.lde.height = 2 * n;
  cm.lde.width = w;
  const uint32_t lde_shift = mmul(to_mont(3), minv(domain_shift));  // GENERATOR / shift
  cm.sharded = plan && plan->sharded(2 * n);
  cm.nxt.free();
  cm.coef.free();
  if (cm.sharded) {
    cm.blk = plan->blk(2 * n);
    cm.row0 = plan->row0(2 * n);
    cm.coef.reset(n * (size_t)w);
    cm.lde.buf.reset(cm.blk * (size_t)w);
    cm.nxt_row0 = (size_t)plan->k2 * cm.blk;  // = row0 for G = 2
    const bool nx = next_cols && !next_cols->empty() && plan->G >= 4;
    if (nx) {
      cm.nxt.reset(cm.blk * next_cols->size());
      cm.nmap.fill(0);  // columns not read at the next row: any valid column
      for (size_t y = 0; y < next_cols->size(); y++) cm.nmap[(*next_cols)[y]] = (uint8_t)y;
    }
    const size_t len = n >> plan->lg;  // the coefficient range this rank opens (open_ood)
    hipEvent_t b0 = timed ? tm->begin(st) : nullptr;
    // iDFT + folds in one pass over the coefficients (the fold time counts as iDFT here)
    int dft_low = -1;
    if (coef_fold_residues(evals, n, w, cm.coef.p, (size_t)plan->k * len, len, lde_shift,
                           plan->lg, plan->r, cm.lde.buf.p, nx ? next_cols : nullptr, plan->r2,
                           cm.nxt.p, &dft_low, st)) {
      if (timed) tm->end(b0, st, split->idft);
      hipEvent_t b1 = timed ? tm->begin(st) : nullptr;
      residue_dft(cm.lde.buf.p, cm.blk, w, dft_low, st);
      if (nx) residue_dft(cm.nxt.p, cm.blk, (int)next_cols->size(), dft_low, st);
      if (timed) tm->end(b1, st, split->dft);
      return;
    }
    lde_coefficients(evals, n, w, cm.coef.p, st);
    if (timed) tm->end(b0, st, split->idft);
    hipEvent_t b1 = timed ? tm->begin(st) : nullptr;
    coset_residue(cm.coef.p, n, w, lde_shift, plan->lg, plan->r, cm.lde.buf.p, st);
    if (nx) coset_residue_cols(cm.coef.p, n, *next_cols, lde_shift, plan->lg, plan->r2, cm.nxt.p, st);
    if (timed) tm->end(b1, st, split->dft);
    return;
  }
  cm.blk = 2 * n;
  cm.row0 = 0;
  cm.lde.buf.reset(2 * n * (size_t)w);
  hipEvent_t b = nullptr;
  if (tm && tm->on) b = tm->begin(st);
  hipEvent_t bs = timed ? tm->begin(st) : nullptr;
  coset_lde(evals, n, w, lde_shift, cm.lde.buf.p, st);
  if (timed) tm->end(bs, st, split->dft);
  if (tm && tm->on) {
    tm->end(b, st, &times->lde_ms);
    times->lde_bytes += 12.0 * (double)n * w;
    times->lde_elem_stages += 3.0 * (double)n * cm.log_n * w;
    times->lde_calls++;
  }
}

void commit_lde(CMat& cm, const uint32_t* evals, size_t n, int w, uint32_t domain_shift,
                hipStream_t st) {
  lde_into(cm, evals, n, w, domain_shift, st, nullptr, nullptr);
}

// ------------------------------------------------------------------------ setup
// The quotient-roots mailbox of each lane (the API lock is held: see open_impl's gbox).
static Mailbox* roots_boxes() {
  static Mailbox boxes[MAX_LANES];
  return boxes;
}

// The host-side buffers a proof on the calling thread's lane uses -- pinned staging arena, fetch
// and roots mailboxes, the opened-value and proof-tail boxes, the group events -- allocated at
// setup: a first proof that pins them itself spends about a millisecond per buffer.
static void warm_lane_host() {
  lane_host_reserve();
  Lane& ln = lane();
  roots_boxes()[ln.id].reserve(4096);
  for (int g = 0; g < Lane::NGEV; g++)
    if (!ln.gev[g]) HIP_CHECK(hipEventCreateWithFlags(&ln.gev[g], hipEventDisableTiming));
  if (!ln.gbox) {
    ln.gcap = 4096;  // EF values; a proof with more regrows it
    HIP_CHECK(hipHostMalloc(&ln.gbox, ln.gcap * sizeof(EF), hipHostMallocDefault));
  }
  if (!ln.tbox) {
    ln.tcap = (size_t)1 << 18;  // words of the proof tail; a longer tail regrows it
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ln.tbox), ln.tcap * 4, hipHostMallocDefault));
  }
}

std::unique_ptr<ProvingKey> setup(const std::string& src) {
  ResidentScope rs;  // the key lives beside the tables, outside every lane's working set
  warm_lane_host();
  twiddles().ensure(TWIDDLE_LOG_MAX);  // every transform size a proof can use (device-built)
  auto pk = std::make_unique<ProvingKey>();
  pk->program = Program::parse(src);
  hipStream_t st = stream();
  int chips[2] = {CHIP_PROGRAM, CHIP_BYTE};
  std::vector<uint32_t> t[2];
  size_t h[2];
  for (int i = 0; i < 2; i++) h[i] = prep_trace(chips[i], pk->program, t[i]);
  int ord[2] = {0, 1};
  if (h[1] > h[0] || (h[1] == h[0] && std::strcmp(CHIP_INFO[chips[1]].name, CHIP_INFO[chips[0]].name) < 0))
    std::swap(ord[0], ord[1]);
  pk->idx_of_chip.fill(-1);
  pk->prep.mats.resize(2);
  pk->prep_evals.resize(2);
  for (int k = 0; k < 2; k++) {
    const int i = ord[k];
    const int w = CHIP_INFO[chips[i]].prep_w;
    pk->chip_of[k] = chips[i];
    pk->idx_of_chip[chips[i]] = k;
    DBuf<uint32_t> rm(h[i] * w);
    HIP_CHECK(hipMemcpyAsync(rm.p, t[i].data(), t[i].size() * 4, hipMemcpyHostToDevice, st));
    pk->prep_evals[k].reset(h[i] * w);
    transpose_bitrev(rm.p, h[i], w, pk->prep_evals[k].p, st);
    HIP_CHECK(hipStreamSynchronize(st));
    lde_into(pk->prep.mats[k], pk->prep_evals[k].p, h[i], w, ONE, st, nullptr, nullptr);
  }
  pk->prep.commit(st);
  return pk;
}

void upload_host_traces(const int* chips, const uint32_t* const* mats, const size_t* heights,
                        const size_t* widths, size_t n, DeviceTraces& dt, hipStream_t st) {
  dt.chips.clear();
  dt.evals.clear();
  dt.heights.clear();
  bool seen[NUM_CHIPS] = {};
  for (size_t i = 0; i < n; i++) {
    const int c = chips[i];
    if (c < 0 || c >= NUM_CHIPS || seen[c]) throw std::runtime_error("traces: bad or repeated chip id");
    seen[c] = true;
    const size_t h = heights[i];
    const int w = CHIP_INFO[c].main_w;
    if ((size_t)w != widths[i])
      throw std::runtime_error(std::string("traces: width mismatch for ") + CHIP_INFO[c].name);
    // a 1-row trace is legal (the Cpu chip of a one-cycle program, cpu/trace.rs:33): its 2-row
    // LDE's reduced opening joins the FRI layer after the last fold
    if (h < 1 || (h & (h - 1)) || h > ((size_t)1 << 23))
      throw std::runtime_error(std::string("traces: height not a power of two in [1, 2^23] for ") +
                               CHIP_INFO[c].name);
    DBuf<uint32_t> rm(h * w);
    upload_bulk(rm.p, mats[i], h * w * 4, st);
    // KoalaBear words are Montgomery residues < p; a larger word breaks mmul's b < p bound
    if (count_noncanonical(rm.p, h * w, st))
      throw std::runtime_error(std::string("traces: non-canonical field word (>= p) in ") +
                               CHIP_INFO[c].name);
    DBuf<uint32_t> ev(h * w);
    transpose_bitrev(rm.p, h, w, ev.p, st);
    dt.chips.push_back(c);
    dt.evals.push_back(std::move(ev));
    dt.heights.push_back(h);
  }
  if (!seen[0]) throw std::runtime_error("traces: the Cpu chip is required");
}

// ------------------------------------------------------------------------ prove
namespace {
// Timing and host-staging scope of one prove call (or one commit / open call of the split
// MachineProver surface).  Kernel probes and stage events are on only when timing is asked for.
struct ProofScope {
  EvTimer ev;
  StageTimes local;
  StageTimes* tms;
  hipEvent_t e_total = nullptr;
  ProofScope(bool timing, StageTimes* times) : tms(times ? times : &local) {
    ev.on = timing && times;
    if (!ev.on) {  // the probes are process-global: only a timed (single-lane) proof arms them
      for (KernelProbe* p : {&ntt_probe(), &p2_probe(), &open_probe(), &reduce_probe()})
        if (p->on) p->on = false;  // (left armed by a timed proof that failed)
      return;
    }
    ntt_probe().reset();
    ntt_probe().on = true;
    p2_probe().reset();
    p2_probe().on = true;
    open_probe().reset();
    open_probe().on = true;
    reduce_probe().reset();
    reduce_probe().on = true;
    e_total = ev.begin(stream());
  }
  void finish() {  // collects every event of the call into *tms
    if (!ev.on) return;
    ev.end(e_total, stream(), &tms->total);
    ev.collect();
    tms->quotient -= tms->spin;  // the overlap-window spins of a solo share's timed run
    tms->total -= tms->spin;
    KernelProbe& pr = ntt_probe();
    pr.collect();
    pr.on = false;
    tms->ntt_kernel_ms = pr.ms;
    tms->ntt_kernel_bytes = pr.bytes;
    tms->ntt_kernel_launches = pr.launches;
    KernelProbe& p2 = p2_probe();
    p2.collect();
    p2.on = false;
    tms->p2_kernel_ms = p2.ms;
    tms->p2_perms = p2.bytes;
    tms->p2_launches = p2.launches;
    KernelProbe& op = open_probe();
    op.collect();
    op.on = false;
    tms->open_kernel_ms = op.ms;
    tms->open_kernel_bytes = op.bytes;
    tms->open_kernel_launches = op.launches;
    KernelProbe& rp = reduce_probe();
    rp.collect();
    rp.on = false;
    tms->reduce_kernel_ms = rp.ms;
    tms->reduce_kernel_bytes = rp.bytes;
    tms->reduce_kernel_launches = rp.launches;
  }
  ~ProofScope() {  // the pinned upload arena is rewound when the call is done
    (void)hipStreamSynchronize(stream());
    staging_reset();
    if (ev.on)  // disarm only what this scope armed (lanes of untimed proofs read the flags)
      for (KernelProbe* p : {&ntt_probe(), &p2_probe(), &open_probe(), &reduce_probe()}) p->on = false;
  }
};

// MachineProver::commit (prover.rs:209-236): sort by (Reverse(height), name), coset LDE of
// every main trace, one MerkleTreeMmcs commit.  md.dt must hold the traces.
void commit_main_impl(MainData& md, ProofScope& ps, bool fetch_root = true) {
  hipStream_t st = stream();
  DeviceTraces& dt = md.dt;
  const int nc = (int)dt.chips.size();
  md.order.resize(nc);
  for (int i = 0; i < nc; i++) md.order[i] = i;
  std::sort(md.order.begin(), md.order.end(), [&](int a, int b) {
    if (dt.heights[a] != dt.heights[b]) return dt.heights[a] > dt.heights[b];
    return std::strcmp(CHIP_INFO[dt.chips[a]].name, CHIP_INFO[dt.chips[b]].name) < 0;
  });
  md.chip.resize(nc);
  md.hn.resize(nc);
  for (int k = 0; k < nc; k++) {
    md.chip[k] = dt.chips[md.order[k]];
    md.hn[k] = dt.heights[md.order[k]];
  }
  htrace().mark("main commit");
  hipEvent_t e0 = ps.ev.on ? ps.ev.begin(st) : nullptr;
  Span span("commit to main traces");  // (no span of its own in the reference: commit_main)
  const Plan plan = make_plan();
  md.mainr = Round();
  md.mainr.mats.resize(nc);
  LdeSplit split{ps.tms ? &ps.tms->main_idft : nullptr, ps.tms ? &ps.tms->main_dft : nullptr};
  for (int k = 0; k < nc; k++) {
    lde_into(md.mainr.mats[k], dt.evals[md.order[k]].p, md.hn[k], CHIP_INFO[md.chip[k]].main_w, ONE,
             st, &ps.ev, ps.tms, &plan, &chip_next_cols(md.chip[k]).main, ps.tms ? &split : nullptr);
    if (ps.tms) ps.tms->main_cells += (double)md.hn[k] * CHIP_INFO[md.chip[k]].main_w;
  }
  hipEvent_t eh = ps.ev.on ? ps.ev.begin(st) : nullptr;
  htrace().mark("main LDE queued");
  md.mainr.commit(st, fetch_root);
  htrace().mark("main tree queued");
  if (ps.ev.on) ps.ev.end(eh, st, &ps.tms->main_hash);
  md.root_on_host = fetch_root;
  if (ps.ev.on) ps.ev.end(e0, st, &ps.tms->main_commit);
}

std::vector<uint8_t> open_impl(const ProvingKey& pk, MainData& md, Challenger ch,
                               const ProveOptions& opt, ProofScope& ps, Challenger* after = nullptr);

// Sharded chips' quotient values: rank j computed LDE positions [j b, (j+1) b) (b = 2n / G),
// which land in chunk (j b) / n at rows [(j b) mod n, + b) of its 4 columns.  An all-gather of
// the chips' parts completes qv on every rank (the chunk LDEs need whole columns).  One exchange
// = pack (one batched copy, then an event), the all-gather once the event has fired (the stream
// keeps running what was queued after the pack), unpack.
struct QuotXchg {
  std::vector<int> chips;
  std::vector<size_t> off;
  size_t total = 0;
  DBuf<uint32_t> send, recv;
  hipEvent_t ready = nullptr;
  QuotXchg() = default;
  QuotXchg(const QuotXchg&) = delete;
  QuotXchg& operator=(const QuotXchg&) = delete;
  ~QuotXchg() {  // an exchange abandoned by an error between its pack and its all-gather
    if (ready) (void)hipEventDestroy(ready);
  }
};
static uint32_t* quot_part(std::vector<DBuf<uint32_t>>& qv, const std::vector<size_t>& hn,
                           const Plan& plan, int k, int rank) {  // rank's part (chunk column 0)
  const size_t n = hn[k], b = plan.blk(2 * n), t0 = (size_t)rank * b;
  return qv[k].p + (t0 / n) * 4 * n + (t0 % n);
}
static void quot_pack(QuotXchg& x, std::vector<DBuf<uint32_t>>& qv, const std::vector<size_t>& hn,
                      const Plan& plan, hipStream_t st) {
  x.off.assign(x.chips.size(), 0);
  x.total = 0;
  for (size_t i = 0; i < x.chips.size(); i++) {
    x.off[i] = x.total;
    x.total += 4 * plan.blk(2 * hn[x.chips[i]]);
  }
  if (!x.total) return;
  x.send.reset(x.total);
  x.recv.reset(x.total * plan.G);
  std::vector<Copy2D> cp;
  for (size_t i = 0; i < x.chips.size(); i++) {
    const int k = x.chips[i];
    const size_t n = hn[k], b = plan.blk(2 * n);
    cp.push_back({quot_part(qv, hn, plan, k, plan.k), x.send.p + x.off[i], n, b, b, 4});
  }
  copy2d_batch(cp, st);
  HIP_CHECK(hipEventCreateWithFlags(&x.ready, hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(x.ready, st));
}
// overlap (timing runs of a rank's share): where the GPU time of the work queued between the
// pack and this call goes (bench.py subtracts it from the collective's modeled time)
static void quot_exchange(QuotXchg& x, const ShardCtx& sc, double* overlap) {
  if (!x.total) return;
  for (;;) {  // the send buffer is complete; later work stays queued on the stream
    const hipError_t e = hipEventQuery(x.ready);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) HIP_CHECK(e);
  }
  HIP_CHECK(hipEventDestroy(x.ready));
  x.ready = nullptr;
  sc.pending_overlap = overlap;
  sc.allgather(x.send.p, x.total * 4, x.recv.p);
  sc.pending_overlap = nullptr;
}
static void quot_unpack(QuotXchg& x, std::vector<DBuf<uint32_t>>& qv,
                        const std::vector<size_t>& hn, const Plan& plan, hipStream_t st) {
  if (!x.total) return;
  std::vector<Copy2D> cp;
  for (int j = 0; j < plan.G; j++)
    for (size_t i = 0; i < x.chips.size(); i++)
      if (j != plan.k) {
        const int k = x.chips[i];
        const size_t n = hn[k], b = plan.blk(2 * n);
        cp.push_back({x.recv.p + (size_t)j * x.total + x.off[i], quot_part(qv, hn, plan, k, j), b,
                      n, b, 4});
      }
  copy2d_batch(cp, st);
  x.send.free();
}
}  // namespace

void commit_main(MainData& md) {
  ProofScope ps(false, nullptr);
  commit_main_impl(md, ps);
  HIP_CHECK(hipStreamSynchronize(stream()));
}

std::vector<uint8_t> open_main(const ProvingKey& pk, MainData& md, const Challenger& ch,
                               const ProveOptions& opt, Challenger* after) {
  ProofScope ps(false, nullptr);
  return open_impl(pk, md, ch, opt, ps, after);
}

Challenger challenger_after_pk(const ProvingKey& pk) {
  Challenger ch;
  ch.observe_digest(pk.prep.tree.root);  // observe_into (prover.rs:595-601): commit + 7 zeros
  for (int i = 0; i < 7; i++) ch.observe(0);
  return ch;
}

std::vector<uint8_t> prove_device(const ProvingKey& pk, DeviceTraces& dt, const ProveOptions& opt,
                                  StageTimes* times) {
  ProofScope ps(opt.timing, times);
  MainData md;
  md.dt = std::move(dt);
  commit_main_impl(md, ps, /*fetch_root=*/false);  // the LogUp challenges are sampled on the device
  auto proof = open_impl(pk, md, challenger_after_pk(pk), opt, ps);
  htrace().mark("open returned");
  ps.finish();
  dt = std::move(md.dt);
  return proof;
}

namespace {
// MachineProver::open (prover.rs:242-553) on the challenger state after pk.observe_into (the
// reference opens on a clone of it, prover.rs:578): observe the main commit, LogUp, quotient,
// PCS open, FRI, grind, queries, BFZ1 serialization.
std::vector<uint8_t> open_impl(const ProvingKey& pk, MainData& md, Challenger ch,
                               const ProveOptions& opt, ProofScope& ps, Challenger* after) {
  hipStream_t st = stream();
  EvTimer& ev = ps.ev;
  StageTimes* tms = ps.tms;
  DeviceTraces& dt = md.dt;
  const std::vector<int>& order = md.order;
  const std::vector<int>& chip = md.chip;
  const std::vector<size_t>& hn = md.hn;
  Round& mainr = md.mainr;
  const int nc = (int)chip.size();
  const Plan plan = make_plan();
  const ShardCtx* shard = shard_ctx();

  // ---- open (prover.rs:242-553), on a clone of the challenger (prover.rs:578)
  htrace().mark("open start");
  // The transcript steps up to zeta run on the device (challenger.h): the LogUp challenges after
  // the main root and the quotient challenge after the permutation root, so neither stage waits
  // for a host round trip.  The host fetches the three roots and the cumulative sums once, after
  // the quotient commit, and replays the same steps before sampling zeta.
  DBuf<DevChallenger> dc_d(1);
  {
    DevChallenger dc;
    std::memcpy(dc.st, ch.st, sizeof(dc.st));
    std::memcpy(dc.in, ch.in, sizeof(dc.in));
    std::memcpy(dc.out, ch.out, sizeof(dc.out));
    dc.nin = ch.nin;
    dc.nout = ch.nout;
    // fault injection for tests/test_gpu.py: a device sponge that is not the host's must end in
    // an error at proving time, not in a proof the verifier rejects
    if (opt.fault_device_challenger)
      dc.st[15] = dc.st[15] ? dc.st[15] - 1 : 1;  // a capacity word (the rate is overwritten)
    upload_async(dc_d.p, &dc, sizeof(dc), st);
  }
  DBuf<PermChallenges> pc_d(1);
  challenge_perm(dc_d.p, mainr.tree.layers.back().p, pc_d.p, st);  // prover.rs:265-272
  htrace().mark("perm challenges");

  hipEvent_t e1 = ev.on ? ev.begin(st) : nullptr;
  Span span("generate permutation traces");  // prover.rs:281 (rows, then each chip's LDE)
  Round permr;
  permr.mats.resize(nc);
  // cums_d: the chips' cumulative sums, then (fetched together) the main, permutation and
  // quotient roots, 2 EF slots (8 words) each, then the device's samples of the LogUp alpha,
  // beta, the quotient alpha and (single GPU) zeta -- compared with the host replay below
  DBuf<EF> cums_d(nc + 10);
  HIP_CHECK(hipMemcpyAsync(cums_d.p + nc, mainr.tree.layers.back().p, 32, hipMemcpyDeviceToDevice, st));
  HIP_CHECK(hipMemcpyAsync(cums_d.p + nc + 6, &pc_d.p->alpha, sizeof(EF), hipMemcpyDeviceToDevice, st));
  HIP_CHECK(hipMemcpyAsync(cums_d.p + nc + 7, &pc_d.p->beta_pows[1], sizeof(EF), hipMemcpyDeviceToDevice, st));
  for (int k = 0; k < nc; k++) {
    const int c = chip[k];
    const int pw = perm_width(c);
    DBuf<uint32_t> pe(4 * (size_t)pw * hn[k]);
    const int pi = pk.idx_of_chip[c];
    const uint32_t* prep = pi >= 0 ? pk.prep_evals[pi].p : nullptr;
    if (k == 0) htrace().mark("perm_rows buffers");
    hipEvent_t br = ev.on ? ev.begin(st) : nullptr;
    perm_trace(c, dt.evals[order[k]].p, prep, hn[k], pc_d.p, pe.p, cums_d.p + k, st);
    if (ev.on) ev.end(br, st, &tms->perm_rows);
    if (k == 0) htrace().mark("perm_rows launched");
    LdeSplit split{tms ? &tms->perm_idft : nullptr, tms ? &tms->perm_dft : nullptr};
    if (tms) tms->perm_cells += (double)hn[k] * 4 * pw;
    lde_into(permr.mats[k], pe.p, hn[k], 4 * pw, ONE, st, &ev, tms, &plan, &chip_next_cols(c).perm,
             tms ? &split : nullptr);
  }
  hipEvent_t bh = ev.on ? ev.begin(st) : nullptr;
  span.begin("commit to permutation traces");  // prover.rs:333
  permr.commit(st, /*fetch_root=*/false);
  span.end();
  if (ev.on) ev.end(bh, st, &tms->perm_hash);
  if (ev.on) ev.end(e1, st, &tms->perm);
  HIP_CHECK(hipMemcpyAsync(cums_d.p + nc + 2, permr.tree.layers.back().p, 32, hipMemcpyDeviceToDevice, st));

  // ---- quotient (prover.rs:344-412)
  hipEvent_t e2 = ev.on ? ev.begin(st) : nullptr;
  span.begin("compute quotient values");  // prover.rs:355 (values, then the chunk LDEs)
  Round quotr;
  quotr.mats.resize(2 * nc);
  std::vector<DBuf<EF>> apows(nc);
  std::vector<QuotParams> qph(nc);  // the challenge-independent fields; the rest on the device
  DBuf<QuotParams> qp_d(std::max(nc, 1));
  QuotAlphaTargets tg{};
  tg.alpha_out = cums_d.p + nc + 8;
  for (int k = 0; k < nc; k++) {
    const size_t n = hn[k];
    const int K = num_constraints(chip[k]);
    apows[k].reset(K);
    tg.apows[k] = apows[k].p;
    tg.K[k] = K;
    QuotParams& qp = qph[k];
    qp.alpha_pows = apows[k].p;
    const uint32_t three = to_mont(3);
    const uint32_t sn = mpow(three, n);
    qp.zh_even = msub(sn, ONE);
    qp.zh_odd = msub(mneg(sn), ONE);
    qp.zh_even_inv = minv(qp.zh_even);
    qp.zh_odd_inv = minv(qp.zh_odd);
    qp.wn_inv = minv(two_adic_gen(log2i(n)));
    qp.shift = three;
  }
  upload_async(qp_d.p, qph.data(), nc * sizeof(QuotParams), st);
  challenge_quot(dc_d.p, permr.tree.layers.back().p, cums_d.p, nc, pc_d.p, qp_d.p, tg, st);
  htrace().mark("quotient challenge");
  std::vector<DBuf<uint32_t>> qv(nc);  // Q on 3 H_2n: 2 chunks x 4 columns of n rows
  auto quot_chip = [&](int k) {
    const int c = chip[k];
    const size_t n = hn[k];
    const int logn = log2i(n);
    const uint32_t three = to_mont(3);
    const QuotParams& qp = qph[k];
    const int pi = pk.idx_of_chip[c];
    const uint32_t* prep_lde = pi >= 0 ? pk.prep.mats[pi].lde.buf.p : nullptr;
    const CMat& mm = mainr.mats[k];
    const CMat& pm = permr.mats[k];
    if (k == 0) htrace().mark("quotient launch");
    if (!mm.sharded) {
      // Chunk cc's domain 3 w_2n^cc H_n is one half of its LDE domain 3 H_2n: the kernel writes
      // each chunk straight into that half of the chunk's LDE buffer (rows [cc n, (cc+1) n))
      // and only the other half is computed below (coset_lde_ex).
      const uint32_t w2n = two_adic_gen(logn + 1);
      for (int cc = 0; cc < 2; cc++) {
        CMat& qm = quotr.mats[2 * k + cc];
        qm.n = n;
        qm.log_n = logn;
        qm.shift = mmul(three, cc ? w2n : ONE);  // split_domains: shift * g^cc
        qm.lde.height = 2 * n;
        qm.lde.width = 4;
        qm.lde.buf.reset(8 * n);
        qm.sharded = false;
        qm.blk = 2 * n;
        qm.row0 = 0;
        qm.coef.free();
        qm.nxt.free();
        for (int j = 0; j < 64; j++) qm.nmap[j] = (uint8_t)j;
      }
      const size_t N = 2 * n;
      QuotRows in{mm.lde.buf.p, mm.lde.buf.p, pm.lde.buf.p, pm.lde.buf.p, prep_lde, N, 0, N, {}, {}};
      for (int j = 0; j < 64; j++) in.nmain[j] = in.nperm[j] = (uint8_t)j;
      quotient_into(c, in, logn + 1, qp,
                    QuotOut{{quotr.mats[2 * k].lde.buf.p, quotr.mats[2 * k + 1].lde.buf.p + n}, N}, st,
                    qp_d.p + k);
      return;
    }
    // sharded: this rank's points only; next rows from the next-residue shards
    qv[k].reset(8 * n);
    QuotRows in{mm.rows(), mm.next_rows(), pm.rows(), pm.next_rows(), prep_lde,
                mm.stride(), mm.row0, mm.blk, {}, {}};
    std::copy(mm.nmap.begin(), mm.nmap.end(), in.nmain);
    std::copy(pm.nmap.begin(), pm.nmap.end(), in.nperm);
    quotient_rows(c, in, logn + 1, qp, qv[k].p, st, qp_d.p + k);
  };
  auto chunk_ldes = [&](int k) {
    const size_t n = hn[k];
    const uint32_t w2n = two_adic_gen(log2i(n) + 1);
    if (!mainr.mats[k].sharded) {  // the other half of each chunk LDE
      for (int cc = 0; cc < 2; cc++) {
        CMat& qm = quotr.mats[2 * k + cc];
        const uint32_t lde_shift = mmul(to_mont(3), minv(qm.shift));  // GENERATOR / shift
        hipEvent_t b = ev.on ? ev.begin(st) : nullptr;
        coset_lde_ex(qm.lde.buf.p + (size_t)cc * n, 2 * n, n, 4, lde_shift, qm.lde.buf.p, 1 - cc, st);
        if (ev.on) {
          ev.end(b, st, &tms->lde_ms);
          tms->lde_bytes += 8.0 * (double)n * 4;  // read n, write n
          tms->lde_elem_stages += 2.0 * (double)n * qm.log_n * 4;
          tms->lde_calls++;
        }
      }
      return;
    }
    for (int cc = 0; cc < 2; cc++) {
      const uint32_t dshift = mmul(to_mont(3), cc ? w2n : ONE);  // split_domains: shift * g^cc
      lde_into(quotr.mats[2 * k + cc], qv[k].p + (size_t)4 * cc * n, n, 4, dshift, st, &ev, tms,
               &plan);
    }
  };
  auto free_next = [&] {  // the next-row shards are done with
    for (int k = 0; k < nc; k++) {
      mainr.mats[k].nxt.free();
      permr.mats[k].nxt.free();
    }
  };
  // Sharded: two exchanges -- every sharded chip but the tallest, then the tallest -- so the first
  // all-gather runs while the GPU computes the tallest chip's quotient and the second while it
  // runs the other chips' chunk LDEs (the collectives are host calls; the stream keeps working
  // through what was queued before them).  BFZ_QUOT_PIPE=0: one exchange after every kernel.
  static const bool pipe = [] {
    const char* e = std::getenv("BFZ_QUOT_PIPE");
    return !(e && *e == '0');
  }();
  int big = -1;
  if (plan.on())
    for (int k = 0; k < nc; k++)
      if (mainr.mats[k].sharded && (big < 0 || hn[k] > hn[big])) big = k;
  if (big < 0) {  // one GPU, or no sharded chip
    for (int k = 0; k < nc; k++) quot_chip(k);
    free_next();
    for (int k = 0; k < nc; k++) chunk_ldes(k);
  } else if (!pipe) {
    for (int k = 0; k < nc; k++) quot_chip(k);
    QuotXchg x;
    for (int k = 0; k < nc; k++)
      if (mainr.mats[k].sharded) x.chips.push_back(k);
    quot_pack(x, qv, hn, plan, st);
    quot_exchange(x, *shard, nullptr);
    quot_unpack(x, qv, hn, plan, st);
    free_next();
    for (int k = 0; k < nc; k++) chunk_ldes(k);
  } else {
    // overlap slots (timing runs of a solo share only): filled when the proof's events resolve
    auto slot = [&]() -> double* {
      if (!ev.on || !shard->solo) return nullptr;
      shard->overlap_store.push_back(0.0);
      return &shard->overlap_store.back();
    };
    QuotXchg xa, xb;
    for (int k = 0; k < nc; k++)
      if (k != big) {
        quot_chip(k);
        if (mainr.mats[k].sharded) xa.chips.push_back(k);
      }
    quot_pack(xa, qv, hn, plan, st);
    double* w1 = slot();
    // timed runs: the window's work is queued behind a 2 ms spin, so it runs back to back as in a
    // real run (queued before the blocking collective) and its span is its GPU time
    if (w1) {
      hipEvent_t sb = ev.begin(st);
      gpu_delay(2000.0, st);
      ev.end(sb, st, &tms->spin);
    }
    hipEvent_t b1 = w1 ? ev.begin(st) : nullptr;
    quot_chip(big);
    xb.chips.push_back(big);
    quot_pack(xb, qv, hn, plan, st);
    if (w1) ev.end(b1, st, w1);
    free_next();
    quot_exchange(xa, *shard, w1);
    quot_unpack(xa, qv, hn, plan, st);
    double* w2 = slot();
    if (w2) {
      hipEvent_t sb = ev.begin(st);
      gpu_delay(2000.0, st);
      ev.end(sb, st, &tms->spin);
    }
    hipEvent_t b2 = w2 ? ev.begin(st) : nullptr;
    for (int k = 0; k < nc; k++)
      if (k != big) chunk_ldes(k);
    if (w2) ev.end(b2, st, w2);
    quot_exchange(xb, *shard, w2);
    quot_unpack(xb, qv, hn, plan, st);
    chunk_ldes(big);
  }
  qv.clear();
  span.begin("commit to quotient traces");  // prover.rs:410
  quotr.commit(st, /*fetch_root=*/false);
  span.end();
  if (ev.on) ev.end(e2, st, &tms->quotient);
  HIP_CHECK(hipMemcpyAsync(cums_d.p + nc + 4, quotr.tree.layers.back().p, 32, hipMemcpyDeviceToDevice, st));
  // Single GPU: zeta is sampled on the device too (prover.rs:415), so the openings below are
  // queued behind the quotient commit with no host round trip; the host reads the roots and the
  // device's samples back through a mailbox while the GPU works, replays the transcript and fails
  // on any mismatch before it uses anything that depends on them.
  const bool dev_zeta = !plan.on();
  EF* const zeta_d = cums_d.p + nc + 9;
  if (dev_zeta) challenge_zeta(dc_d.p, quotr.tree.layers.back().p, zeta_d, st);
  Mailbox& roots_box = roots_boxes()[lane().id];
  roots_box.post(cums_d.p, (nc + 10) * sizeof(EF), st);
  EF zeta = ef_zero();
  std::vector<EF> cums(nc + 10);  // [0, nc): the chips' cumulative sums (written into the proof)
  auto replay = [&] {
    roots_box.wait(cums.data(), (nc + 10) * sizeof(EF));
    htrace().mark("roots fetched");
    std::memcpy(mainr.tree.root, &cums[nc], 32);
    std::memcpy(permr.tree.root, &cums[nc + 2], 32);
    std::memcpy(quotr.tree.root, &cums[nc + 4], 32);
    md.root_on_host = true;
    // The host transcript replays the device steps (prover.rs:265-272, 336-342, 413-416): the
    // reference has one transcript, so the device's samples must be the host's (a drifted device
    // sponge would otherwise surface only as a proof the verifier rejects).
    auto same = [](const EF& dev, const EF& host, const char* what) {
      if (!ef_eq(dev, host))
        throw std::runtime_error(std::string("device transcript diverged from the host challenger: ") + what);
    };
    ch.observe_digest(mainr.tree.root);
    same(cums[nc + 6], ch.sample_ef(), "LogUp alpha");
    same(cums[nc + 7], ch.sample_ef(), "LogUp beta");
    ch.observe_digest(permr.tree.root);
    for (int k = 0; k < nc; k++) ch.observe_ef(cums[k]);
    same(cums[nc + 8], ch.sample_ef(), "quotient alpha");
    ch.observe_digest(quotr.tree.root);
    zeta = ch.sample_ef();
    if (dev_zeta) same(cums[nc + 9], zeta, "zeta");
    htrace().mark("zeta");
  };
  if (!dev_zeta) replay();

  // ---- PCS open: opened values (prover.rs:417-470)
  hipEvent_t e3 = ev.on ? ev.begin(st) : nullptr;
  span.begin("open multi batches");  // prover.rs:460 (opened values, reduced openings, FRI, queries)
  const Round* rounds[4] = {&pk.prep, &mainr, &permr, &quotr};
  struct MatPts {
    int npts;
    EF pts[2];
    size_t off[2];  // offsets into the opened-values buffer
  };
  std::vector<MatPts> mp[4];
  int Lmax = 0;
  size_t nvals = 0;
  for (int r = 0; r < 4; r++) {
    for (size_t i = 0; i < rounds[r]->mats.size(); i++) {
      const CMat& m = rounds[r]->mats[i];
      bool lo;
      if (r == 0) lo = CHIP_INFO[pk.chip_of[i]].local_only;
      else if (r == 1) lo = CHIP_INFO[chip[i]].local_only;
      else lo = (r == 3);
      MatPts p;
      p.npts = lo ? 1 : 2;
      p.pts[0] = zeta;
      p.pts[1] = ef_mul_base(zeta, two_adic_gen(m.log_n));
      for (int j = 0; j < p.npts; j++) {
        p.off[j] = nvals;
        nvals += m.lde.width;
      }
      mp[r].push_back(p);
      Lmax = std::max(Lmax, m.log_n + LOG_BLOWUP);
    }
  }
  // Inverse denominators 1 / (x_t - point), indexed by global LDE position.  Unsharded: one
  // table over the tallest height for zeta (smaller heights read its prefix) and one per height
  // for the second point.  Sharded: per height, the rank's range where the height is sharded
  // and the whole height where it is replicated.
  // A replicated matrix at a sharded height (the preprocessed ones) is opened over its whole
  // low coset: that height also gets full tables (fa, fb).
  struct Invd {
    DBuf<EF> a, b, fa, fb;
    size_t t0 = 0;
    const EF* pa() const { return a.p - t0; }
    const EF* pb() const { return b.p ? b.p - t0 : nullptr; }
    const EF* full_a() const { return fa.p ? fa.p : a.p; }  // a is full where fa is absent
    const EF* full_b() const { return fa.p ? fb.p : b.p; }
  };
  std::map<int, bool> two_at;  // LDE log heights present -> some matrix opened at two points
  std::map<int, bool> rep_at;  // ... -> a replicated matrix is opened at that height
  for (int r = 0; r < 4; r++)
    for (size_t i = 0; i < rounds[r]->mats.size(); i++) {
      const int lh = rounds[r]->mats[i].log_n + LOG_BLOWUP;
      two_at[lh] |= mp[r][i].npts == 2;
      rep_at[lh] |= !rounds[r]->mats[i].sharded;
    }
  htrace().mark("inv_denoms launch");
  DBuf<EF> invd_zeta, w_zeta;
  static const bool wtab_on = [] {  // BFZ_OPEN_WTAB=0: weights computed in the openings (A/B)
    const char* e = std::getenv("BFZ_OPEN_WTAB");
    return !(e && *e == '0');
  }();
  if (!plan.on()) {
    invd_zeta.reset((size_t)1 << Lmax);
    if (wtab_on) w_zeta.reset((size_t)1 << (Lmax - 1));
    inv_denoms_dev(zeta_d, Lmax, invd_zeta.p, st, w_zeta.p);
  }
  // a sharded proof's many small opening launches (one per matrix, table and height) go out as
  // one batch each (BFZ_OPEN_SHARD_BATCH=0: one launch per matrix / table / range, A/B)
  static const bool sbatch = [] {
    const char* e = std::getenv("BFZ_OPEN_SHARD_BATCH");
    return !(e && *e == '0');
  }();
  std::vector<InvJob> ijobs;
  auto inv_range = [&](const EF& z, int lh, size_t t0, size_t cnt, EF* out) {
    if (sbatch) ijobs.push_back({z, lh, t0, cnt, out});
    else inv_denoms_range(z, lh, t0, cnt, out, st);
  };
  std::map<int, Invd> invd;
  for (const auto& [lh, two] : two_at) {
    const size_t H = (size_t)1 << lh;
    const bool sh = plan.sharded(H);
    const size_t t0 = sh ? plan.row0(H) : 0, cnt = sh ? plan.blk(H) : H;
    Invd& d = invd[lh];
    d.t0 = t0;
    if (plan.on()) {
      d.a.reset(cnt);
      inv_range(zeta, lh, t0, cnt, d.a.p);
    } else {
      d.a = DBuf<EF>::borrow(invd_zeta.p, H);
    }
    const EF znext = ef_mul_base(zeta, two_adic_gen(lh - LOG_BLOWUP));
    if (two && plan.on()) {  // single GPU: read from the zeta table (prev2_pos, fri.hip)
      d.b.reset(cnt);
      inv_range(znext, lh, t0, cnt, d.b.p);
    }
    if (sh && rep_at[lh]) {  // the low coset only: positions [0, H / 2)
      d.fa.reset(H / 2);
      inv_range(zeta, lh, 0, H / 2, d.fa.p);
      if (two) {
        d.fb.reset(H / 2);
        inv_range(znext, lh, 0, H / 2, d.fb.p);
      }
    }
  }
  inv_denoms_ranges(ijobs, st);
  // Opened values.  Replicated matrices: barycentric over the low coset of the LDE.  Sharded
  // matrices: the rank's 1/G slice of sum_j c_j (z / s)^j (s = the trace domain's shift) from
  // the kept coefficients; the slices are summed across ranks below.
  DBuf<EF> opened_d(nvals);
  std::map<std::array<uint32_t, 5>, DBuf<EF>> ptabs;  // (point, log n) -> powers on the range
  std::vector<PowJob> pjobs;
  auto ptable = [&](const EF& z, int log_n, size_t j0, size_t len) {
    const std::array<uint32_t, 5> key{z.c[0], z.c[1], z.c[2], z.c[3], (uint32_t)log_n};
    auto it = ptabs.find(key);
    if (it != ptabs.end()) return (const EF*)it->second.p;
    DBuf<EF> t(len);
    if (sbatch) pjobs.push_back({z, j0, len, t.p});
    else pow_table(z, j0, len, t.p, st);
    const EF* p = t.p;
    ptabs.emplace(key, std::move(t));
    return p;
  };
  // Unsharded: the openings run in three transcript-ordered groups (preprocessed + main rounds,
  // the permutation round, the quotient round), each copied to the host as soon as it is done,
  // so the host observes a group (~250 host permutations in all) while the GPU computes the
  // next one instead of after all of them.
  const bool grouped = !plan.on();
  auto group_of = [&](int r) { return !grouped ? 0 : r <= 1 ? 0 : r - 1; };
  constexpr int NGROUP = 3;
  std::vector<OpenDesc> open1g[NGROUP], open2g[NGROUP];
  size_t gend[NGROUP] = {0, 0, 0};  // end of each group's range in the opened-value buffer
  for (int r = 0; r < 4; r++)
    for (size_t i = 0; i < rounds[r]->mats.size(); i++) {
      const CMat& m = rounds[r]->mats[i];
      const int lh = m.log_n + LOG_BLOWUP;
      const bool two = mp[r][i].npts == 2;
      EF* out_a = opened_d.p + mp[r][i].off[0];
      EF* out_b = two ? opened_d.p + mp[r][i].off[1] : nullptr;
      if (m.sharded) {
        const size_t len = m.n >> plan.lg, j0 = (size_t)plan.k * len;
        const uint32_t sinv = minv(m.shift);
        const EF* tab[2] = {nullptr, nullptr};
        for (int j = 0; j < mp[r][i].npts; j++)
          tab[j] = ptable(ef_mul_base(mp[r][i].pts[j], sinv), m.log_n, j0, len);
        const EF ninv = ef_base(minv(to_mont((uint32_t)(m.n % P))));
        if (!sbatch) {
          open_coefficients(m.coef.p + j0, m.n, m.lde.width, len, tab[0], ninv, out_a, tab[1],
                            ninv, out_b, st);
          continue;
        }
        OpenDesc o{};  // the coefficient form in the batched launch (fri.h)
        o.tab = 1;
        o.mat = m.coef.p + j0;
        o.height = m.n;  // column stride
        o.rows = len;
        o.w = m.lde.width;
        o.logH = lh;
        o.invd_a = tab[0];
        o.invd_b = two ? tab[1] : tab[0];
        o.scale_a = o.scale_b = ninv;
        o.out_a = out_a;
        o.out_b = two ? out_b : out_a;
        (two ? open2g : open1g)[group_of(r)].push_back(o);
        continue;
      }
      const uint32_t three_n = mpow(to_mont(3), m.n);
      const uint32_t n_f = to_mont((uint32_t)(m.n % P));
      const Invd& d = invd.at(lh);
      OpenDesc o{};
      o.mat = m.lde.buf.p;
      o.height = m.lde.height;
      o.w = m.lde.width;
      o.logH = lh;
      o.invd_a = d.full_a();
      o.invd_b = two ? d.full_b() : o.invd_a;  // nullptr: derived from the zeta table
      // scale = (z^n - 3^n) / (3^n n), the same for both points ((zeta w_n)^n = zeta^n); with
      // derived second-point denominators it also carries w_n^-1 (see k_reduce)
      o.wtab = w_zeta.p;  // unsharded: the weight table (nullptr: weights computed per row)
      const uint32_t zb = two && !o.invd_b && !o.wtab ? minv(two_adic_gen(m.log_n)) : ONE;
      if (dev_zeta) {  // computed by k_open_final_batch from the device's zeta
        o.zeta = zeta_d;
        o.zlog = m.log_n;
        o.z3n = three_n;
        o.zc = minv(mmul(three_n, n_f));
        o.zb = zb;
      } else {
        const EF zn = ef_pow(zeta, m.n);
        o.scale_a = ef_mul_base(ef_sub(zn, ef_base(three_n)), minv(mmul(three_n, n_f)));
        o.scale_b = ef_mul_base(o.scale_a, zb);
      }
      o.out_a = out_a;
      o.out_b = two ? out_b : out_a;
      (two ? open2g : open1g)[group_of(r)].push_back(o);
    }
  pow_tables(pjobs, st);  // before the opening batches that read them (same stream)
  for (int r = 0; r < 4; r++)
    if (!mp[r].empty()) {
      const MatPts& last = mp[r].back();
      gend[group_of(r)] = std::max(gend[group_of(r)], last.off[last.npts - 1] +
                                                          rounds[r]->mats.back().lde.width);
    }
  std::vector<EF> opened(nvals);
  // gev / gbox (and tbox below) belong to this proof's lane and are reallocated on the
  // assumption that no copy into them is pending: safe only because every caller holds the API
  // lock (one proof per lane at a time) and every proof synchronizes before it returns.  A
  // caller outside the lock is a bug.
  if (api_lock_depth() == 0) throw std::logic_error("open_impl called outside the bfz API lock");
  static_assert(NGROUP <= Lane::NGEV, "lane events");
  Lane& ln = lane();
  hipEvent_t* gev = ln.gev;
  if (grouped) {
    if (!gev[0])
      for (int g = 0; g < NGROUP; g++) HIP_CHECK(hipEventCreateWithFlags(&gev[g], hipEventDisableTiming));
    if (nvals > ln.gcap) {  // no copy into it is pending: every proof waits for its groups
      if (ln.gbox) HIP_CHECK(hipHostFree(ln.gbox));
      ln.gcap = std::max(nvals, (size_t)1024);
      HIP_CHECK(hipHostMalloc(&ln.gbox, ln.gcap * sizeof(EF), hipHostMallocDefault));
    }
  }
  EF* gbox = static_cast<EF*>(ln.gbox);
  for (int g = 0; g < (grouped ? NGROUP : 1); g++) {
    open_batch(open2g[g], 2, st);  // barycentric openings: two partial + two final launches
    open_batch(open1g[g], 1, st);
    if (!grouped) break;
    const size_t b0 = g ? gend[g - 1] : 0, b1 = std::max(gend[g], b0);
    if (b1 > b0)
      HIP_CHECK(hipMemcpyAsync(gbox + b0, opened_d.p + b0, (b1 - b0) * sizeof(EF),
                               hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipEventRecord(gev[g], st));
  }
  // ---- reduced-opening descriptors (TwoAdicFriPcs::open, prover.rs:460-470), built while the
  // openings run: per LDE height, every column of every matrix opened there in round order; the
  // alpha-dependent parts (column coefficients alpha^k, the matrices' alpha^w, the job's ya / yb)
  // are filled by reduce_prep on the device once alpha is known, so the host's work after the
  // last opened value is observing it and sampling alpha.
  struct RedJob {
    int lh;
    size_t col0, mat0, ncols;
    int nmats;
    bool has_b;
  };
  std::vector<RedCol> red_cols;
  std::vector<RedMat> red_mats;
  std::vector<RedJob> red_jobs;
  std::vector<RedColPrep> col_prep;
  std::vector<RedMatPrep> mat_prep;
  std::vector<RedJobPrep> job_prep;
  for (int lh = Lmax; lh >= 1; lh--) {
    const size_t col0 = red_cols.size(), mat0 = red_mats.size();
    uint32_t e = 0;  // the reduction order: point a's columns, then point b's, matrix by matrix
    bool has_b = false;
    for (int r = 0; r < 4; r++)
      for (size_t i = 0; i < rounds[r]->mats.size(); i++) {
        const CMat& m = rounds[r]->mats[i];
        if (m.log_n + LOG_BLOWUP != lh) continue;
        const int w = m.lde.width;
        const bool two = mp[r][i].npts == 2;
        RedMat rm{};
        rm.first = (int)(red_cols.size() - col0);
        rm.count = w;
        rm.has_b = two ? 1 : 0;
        for (int c = 0; c < w; c++) {
          RedCol rc{};
          rc.col = m.rows() + (size_t)c * m.stride();
          red_cols.push_back(rc);
          col_prep.push_back({e + (uint32_t)c, (uint32_t)(mp[r][i].off[0] + c),
                              two ? (uint32_t)(mp[r][i].off[1] + c) : 0xffffffffu, (uint32_t)w});
        }
        // the second point's coefficients are the first point's times alpha^w; single GPU: its
        // denominators come from the zeta table times w_n^-1 (reduce_range), folded into kb / yb
        mat_prep.push_back({(uint32_t)w, two && !plan.on() ? minv(two_adic_gen(m.log_n)) : ONE});
        red_mats.push_back(rm);
        e += (uint32_t)(mp[r][i].npts * w);
        has_b |= two;
      }
    if (red_cols.size() == col0) continue;
    const size_t ncols = red_cols.size() - col0, nm = red_mats.size() - mat0;
    red_jobs.push_back({lh, col0, mat0, ncols, (int)nm, has_b});
    RedJobPrep jp{};
    jp.col0 = (uint32_t)col0;
    jp.ncols = (uint32_t)ncols;
    jp.mat0 = (uint32_t)mat0;
    jp.nmats = (uint32_t)nm;
    jp.yb_fold = has_b && !plan.on() ? minv(two_adic_gen(lh - LOG_BLOWUP)) : ONE;
    job_prep.push_back(jp);
  }
  DBuf<RedCol> red_cols_d(std::max<size_t>(red_cols.size(), 1));
  DBuf<RedMat> red_mats_d(std::max<size_t>(red_mats.size(), 1));
  DBuf<RedColPrep> col_prep_d(std::max<size_t>(col_prep.size(), 1));
  DBuf<RedMatPrep> mat_prep_d(std::max<size_t>(mat_prep.size(), 1));
  DBuf<RedJobPrep> job_prep_d(std::max<size_t>(job_prep.size(), 1));
  upload_async(red_cols_d.p, red_cols.data(), red_cols.size() * sizeof(RedCol), st);
  upload_async(red_mats_d.p, red_mats.data(), red_mats.size() * sizeof(RedMat), st);
  upload_async(col_prep_d.p, col_prep.data(), col_prep.size() * sizeof(RedColPrep), st);
  upload_async(mat_prep_d.p, mat_prep.data(), mat_prep.size() * sizeof(RedMatPrep), st);
  upload_async(job_prep_d.p, job_prep.data(), job_prep.size() * sizeof(RedJobPrep), st);
  htrace().mark("reduce descriptors");

  if (dev_zeta) replay();  // the openings are queued: now the host's transcript catches up
  if (plan.on()) {  // one all-gather; sharded matrices' slices summed, replicated ones kept
    DBuf<EF> all(nvals * plan.G);
    coll_sync(st);
    htrace().mark("sharded openings done");
    shard->allgather(opened_d.p, nvals * sizeof(EF), all.p);
    std::vector<EF> h(nvals * plan.G);
    HIP_CHECK(hipMemcpyAsync(h.data(), all.p, h.size() * sizeof(EF), hipMemcpyDeviceToHost, st));
    coll_sync(st);
    htrace().mark("sharded openings on host");
    for (int r = 0; r < 4; r++)
      for (size_t i = 0; i < rounds[r]->mats.size(); i++) {
        const CMat& m = rounds[r]->mats[i];
        for (int j = 0; j < mp[r][i].npts; j++)
          for (int c = 0; c < m.lde.width; c++) {
            const size_t o = mp[r][i].off[j] + c;
            EF v = h[(size_t)plan.k * nvals + o];
            if (m.sharded) {
              v = ef_zero();
              for (int g = 0; g < plan.G; g++) v = ef_add(v, h[(size_t)g * nvals + o]);
            }
            opened[o] = v;
          }
      }
  }
  // the opened values reduce_prep reads: the openings' own buffer (single GPU) or, sharded, the
  // rank-summed values assembled above
  DBuf<EF> opened_sum_d;
  const EF* opened_dev = opened_d.p;
  if (plan.on()) {
    opened_sum_d.reset(std::max<size_t>(nvals, 1));
    upload_async(opened_sum_d.p, opened.data(), nvals * sizeof(EF), st);
    opened_dev = opened_sum_d.p;
  }
  auto wait_group = [&](int g) {  // the group's values in `opened`
    for (;;) {
      const hipError_t e = hipEventQuery(gev[g]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) HIP_CHECK(e);
    }
    const size_t b0 = g ? gend[g - 1] : 0, b1 = std::max(gend[g], b0);
    std::copy(gbox + b0, gbox + b1, opened.begin() + b0);
  };
  if (grouped) {
    int have = -1;  // groups copied into `opened` so far
    for (int r = 0; r < 4; r++) {
      while (have < group_of(r)) wait_group(++have);
      if (opt.observe_openings)  // decision D1: opened values enter the transcript
        for (size_t i = 0; i < rounds[r]->mats.size(); i++)
          for (int j = 0; j < mp[r][i].npts; j++)
            for (int c = 0; c < rounds[r]->mats[i].lde.width; c++)
              ch.observe_ef(opened[mp[r][i].off[j] + c]);
    }
    while (have < NGROUP - 1) wait_group(++have);
    htrace().mark("opened observed");
  } else if (opt.observe_openings) {
    htrace().mark("opened summed");
    for (int r = 0; r < 4; r++)
      for (size_t i = 0; i < rounds[r]->mats.size(); i++)
        for (int j = 0; j < mp[r][i].npts; j++)
          for (int c = 0; c < rounds[r]->mats[i].lde.width; c++)
            ch.observe_ef(opened[mp[r][i].off[j] + c]);
  }
  const EF fri_alpha = ch.sample_ef();
  htrace().mark("fri alpha");

  // ---- reduced openings: the alpha-dependent coefficients of the descriptors built above, then
  // one k_reduce launch per LDE height
  DBuf<EF> alpha_yab(1 + 2 * std::max<size_t>(red_jobs.size(), 1));  // alpha, then {ya, yb} per job
  upload_async(alpha_yab.p, &fri_alpha, sizeof(EF), st);
  reduce_prep(red_cols_d.p, col_prep_d.p, red_mats_d.p, mat_prep_d.p, job_prep_d.p,
              (int)red_jobs.size(), opened_dev, alpha_yab.p, alpha_yab.p + 1, st);
  std::map<int, DBuf<EF>> ro;
  for (size_t ji = 0; ji < red_jobs.size(); ji++) {
    const RedJob& j = red_jobs[ji];
    const size_t H = (size_t)1 << j.lh;
    const bool sh = plan.sharded(H);
    const size_t t0 = sh ? plan.row0(H) : 0, cnt = sh ? plan.blk(H) : H;
    DBuf<EF> r(cnt);
    const Invd& d = invd.at(j.lh);
    reduce_range(red_cols_d.p + j.col0, red_mats_d.p + j.mat0, j.nmats, H, t0, cnt, d.pa(),
                 j.has_b ? d.pb() : nullptr, alpha_yab.p + 1 + 2 * ji, j.has_b, r.p - t0, st,
                 (int)j.ncols);
    ro.emplace(j.lh, std::move(r));
  }
  if (ev.on) ev.end(e3, st, &tms->open);

  // ---- FRI commit phase (fri::prover::commit_phase)
  hipEvent_t e4 = ev.on ? ev.begin(st) : nullptr;
  // A layer of a sharded proof stays row-sharded (values [e0, e0 + len / G)) while its fold
  // output has >= G * 1024 values; the first shorter one is all-gathered and the rest is
  // computed by every rank.
  struct FriLayer {
    DBuf<EF> v;
    size_t e0 = 0;
    bool local = false;
  };
  std::vector<FriLayer> layers;
  std::vector<MerkleTree> trees;
  {
    const size_t H = (size_t)1 << Lmax;
    layers.push_back({std::move(ro.at(Lmax)), plan.sharded(H) ? plan.row0(H) : 0, plan.sharded(H)});
  }
  ro.erase(Lmax);
  // The transcript steps of the rounds run on the device (fri_challenge): the input buffer is
  // empty here (fri_alpha was just sampled), so each round is observe(root) -> one duplex ->
  // beta = 4 pops, and no host round trip is needed until the final polynomial.
  if (ch.nin != 0) throw std::runtime_error("FRI: unexpected pending challenger input");
  DBuf<uint32_t> dstate(16);
  upload_async(dstate.p, ch.st, 64, st);
  const int nrounds = Lmax - LOG_BLOWUP;
  DBuf<EF> betas(std::max(nrounds, 1));
  size_t len = (size_t)1 << Lmax;
  // Every sharded round costs one subtree-root all-gather: rounds stay sharded only while
  // h >= FRI_SHARD_MIN and the shorter tail (a few hundred thousand permutations) runs on every
  // rank after one all-gather of the layer.
  // (BFZ_FRI_SHARD_MIN overrides it: the tests shard small proofs' rounds too)
  static const size_t FRI_SHARD_MIN = [] {
    const char* e = std::getenv("BFZ_FRI_SHARD_MIN");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)1 << 18;
  }();
  auto fri_sharded = [&](size_t h) { return plan.sharded(h) && h >= FRI_SHARD_MIN; };
  auto gather = [&](DBuf<EF>& v, size_t len) {  // a row-sharded vector of len values, in place
    DBuf<EF> all(len);
    coll_sync(st);
    shard->allgather(v.p, plan.blk(len) * sizeof(EF), all.p);
    v = std::move(all);
  };
  DBuf<uint32_t> tail_trees;  // the tail rounds' trees and layers (views below borrow them)
  DBuf<EF> tail_layers;
  // A replicated round's fold is left pending and runs fused with the next round's leaf hashes
  // (fri_fold_leaves): layers.back() is then allocated but not yet written.
  struct PendingFold {
    const EF* in = nullptr;
    const EF* beta = nullptr;
    const EF* add = nullptr;
    size_t n = 0;  // fold outputs
  } pend;
  auto flush_fold = [&]() {
    if (!pend.in) return;
    fri_fold_range(pend.in, layers.back().v.p, pend.n, 0, pend.n, pend.beta, pend.add, st);
    pend = PendingFold{};
  };
  for (int rd = 0; len > ((size_t)1 << LOG_BLOWUP); rd++) {
    const size_t h = len / 2;
    FriLayer& cur = layers.back();
    if (!cur.local && h <= (size_t)FRI_TAIL_MAXH) {  // every remaining round in one launch
      flush_fold();
      FriTailRounds a;
      a.logh0 = log2i(h);
      a.nr = log2i(len) - LOG_BLOWUP;
      a.in = cur.v.p;
      a.state = dstate.p;
      a.beta = betas.p + rd;
      size_t nw = 0, nv = 0;
      for (int r = 0; r < a.nr; r++) {
        nw += 8 * ((h >> r) * 2 - 1);
        nv += h >> r;
      }
      tail_trees.reset(nw);
      tail_layers.reset(nv);
      nw = nv = 0;
      for (int r = 0; r < a.nr; r++) {
        const size_t hr = h >> r;
        const EF* rows = r ? tail_layers.p + nv - 2 * hr : cur.v.p;
        trees.emplace_back();
        MerkleTree& t = trees.back();
        t.mats = {MatRef{(const uint32_t*)rows, hr, 8}};
        t.layers.resize(log2i(hr) + 1);
        a.tree[r] = tail_trees.p + nw;
        for (size_t L = 0; L < t.layers.size(); L++) {
          t.layers[L] = DBuf<uint32_t>::borrow(tail_trees.p + nw, 8 * (hr >> L));
          nw += 8 * (hr >> L);
        }
        a.layer[r] = tail_layers.p + nv;
        const int lgh = log2i(hr);
        a.add[r] = ro.count(lgh) ? ro.at(lgh).p : nullptr;
        layers.push_back({DBuf<EF>::borrow(tail_layers.p + nv, hr), 0, false});
        nv += hr;
      }
      fri_tail_rounds(a, st);
      len = h >> (a.nr - 1);
      break;
    }
    if (cur.local && !fri_sharded(h)) {
      gather(cur.v, len);
      cur.e0 = 0;
      cur.local = false;
    }
    const bool loc = cur.local;
    const size_t i0 = loc ? plan.row0(h) : 0, cnt = loc ? plan.blk(h) : h;
    trees.emplace_back();
    MerkleTree& t = trees.back();
    std::function<void(size_t, size_t, uint32_t*)> fused;
    if (pend.in) {  // this round's layer is the pending fold's output: fold + hash in one pass
      const PendingFold pf = pend;
      EF* out = cur.v.p;
      fused = [pf, out, h, &st](size_t, size_t, uint32_t* dig) {
        fri_fold_leaves(pf.in, out, h, pf.beta, pf.add, dig, st);
      };
      pend = PendingFold{};
    }
    merkle_from_rows8(t, (const uint32_t*)(cur.v.p - 2 * i0), h, st, /*fetch_root=*/false,
                      RootChallenge{dstate.p, betas.p + rd}, /*allow_shard=*/loc, fused);
    DBuf<EF> next(cnt);
    const int lgh = log2i(h);
    if (!loc && ro.count(lgh) && plan.sharded(h)) gather(ro.at(lgh), h);  // replicated tail
    const EF* add = ro.count(lgh) ? ro.at(lgh).p : nullptr;  // same range as next
    if (!loc && h / 2 >= FRI_FUSE_MIN) pend = PendingFold{cur.v.p, betas.p + rd, add, h};
    else fri_fold_range(cur.v.p, next.p, h, i0, cnt, betas.p + rd, add, st);
    layers.push_back({std::move(next), i0, loc});
    len = h;
  }
  flush_fold();
  const int nt = (int)trees.size();
  if (nt > MAX_FRI_ROUNDS) throw std::runtime_error("FRI: too many rounds");
  const int nq = opt.num_queries;

  // ---- query openings: every opened word in proof order
  // Opening segments in serialization order (same for every query; see GatherSeg).
  auto owner_shift = [](const MerkleTree& t, int L) {  // layer L of a sharded tree
    const int nl = (int)t.layers.size() - 1;
    return L < t.sharded_below ? nl - L - t.shard_log : -1;
  };
  std::vector<GatherSeg> segs;
  const int ncommit = nt;
  // The segments follow the serialized query layout, its length words included as literal
  // segments (base == nullptr: count words of value xr), so the gathered words are the query
  // section of the proof as is.
  auto lit = [&](uint32_t v) { segs.push_back({nullptr, 0, 0, v, 0, 1, -1, 0}); };
  lit(4);
  for (int r = 0; r < 4; r++) {
    const Round& R = *rounds[r];
    const int lrm = (int)R.tree.layers.size() - 1;
    lit((uint32_t)R.mats.size());
    for (const CMat& m : R.mats) {  // row (index >> (Lmax - lh)) of every column
      const int lh = log2i(m.lde.height);
      lit((uint32_t)m.lde.width);
      segs.push_back({m.rows(), (uint64_t)m.stride(), (uint32_t)(Lmax - lh), 0, 1,
                      (uint32_t)m.lde.width, m.sharded ? lh - plan.lg : -1, 0});
    }
    lit((uint32_t)lrm);
    for (int L = 0; L < lrm; L++)  // sibling digest at layer L
      segs.push_back({R.tree.layers[L].p, 1, (uint32_t)(Lmax - lrm + L), 1, 8, 8,
                      owner_shift(R.tree, L), 0});
  }
  lit((uint32_t)ncommit);
  for (int i = 0; i < ncommit; i++) {
    const FriLayer& fl = layers[i];  // sibling EF
    segs.push_back({(const uint32_t*)(fl.v.p - fl.e0), 1, (uint32_t)i, 1, 4, 4,
                    fl.local ? Lmax - i - plan.lg : -1, 0});
    const int lm = (int)trees[i].layers.size() - 1;
    lit((uint32_t)lm);
    for (int L = 0; L < lm; L++)
      segs.push_back({trees[i].layers[L].p, 1, (uint32_t)(i + 1 + L), 1, 8, 8,
                      owner_shift(trees[i], L), 0});
  }
  const size_t nwords = query_words(segs) * (size_t)nq;

  // ---- the transcript tail on the device: observe the final constant, grind, sample the
  // query indices (fri_transcript_tail), then the gather; one device-to-host copy returns the
  // commit-phase roots, the final layer, the challenger, the witness and the query words.
  // tail = [roots (8 MAX_FRI_ROUNDS) | FRI state (16) | final layer (8) | challenger | witness,
  //         ok | qidx (nq) | query words]
  constexpr size_t T_CH = 8 * MAX_FRI_ROUNDS + 16 + 8;
  constexpr size_t T_RES = T_CH + sizeof(DevChallenger) / 4;
  constexpr size_t T_Q = T_RES + 2;
  static_assert(sizeof(DevChallenger) % 4 == 0, "DevChallenger: whole words");
  const size_t T_W = T_Q + (size_t)nq, tail_n = T_W + nwords;
  DBuf<uint32_t> tailbuf(tail_n);
  DevChallenger* dch = reinterpret_cast<DevChallenger*>(tailbuf.p + T_CH);
  if (!nt) {  // no commit-phase round: the host challenger as it stands
    DevChallenger hc;
    std::memcpy(hc.st, ch.st, 64);
    std::memcpy(hc.in, ch.in, 32);
    std::memcpy(hc.out, ch.out, 32);
    hc.nin = ch.nin;
    hc.nout = ch.nout;
    upload_async(dch, &hc, sizeof(hc), st);
  }
  FriTail tail{};
  for (int i = 0; i < nt; i++) tail.root[i] = trees[i].layers.back().p;
  tail.nroots = nt;
  tail.state = dstate.p;
  tail.fin = layers.back().v.p;
  hipLaunchKernelGGL(k_pack_fri_tail, dim3(1), dim3(256), 0, st, tail, tailbuf.p);
  KCHECK();
  htrace().mark("grind");
  fri_transcript_tail(dch, nt ? dstate.p : nullptr, layers.back().v.p, POW_BITS, nq, Lmax,
                      tailbuf.p + T_Q, tailbuf.p + T_RES, st);
  gather_queries(segs, tailbuf.p + T_Q, nq, tailbuf.p + T_W, shard, st);
  Lane& tl = lane();  // pinned: the tail of the proof (per lane)
  if (tail_n > tl.tcap) {  // no copy into it is pending: every proof waits for its tail
    if (tl.tbox) HIP_CHECK(hipHostFree(tl.tbox));
    tl.tcap = tail_n + tail_n / 4;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&tl.tbox), tl.tcap * 4, hipHostMallocDefault));
  }
  uint32_t* tbox = tl.tbox;
  HIP_CHECK(hipMemcpyAsync(tbox, tailbuf.p, tail_n * 4, hipMemcpyDeviceToHost, st));
  spin_sync(st);
  htrace().mark("queries gathered");
  for (int i = 0; i < nt; i++) std::memcpy(trees[i].root, &tbox[8 * i], 32);
  EF fin[2];
  std::memcpy(fin, &tbox[8 * MAX_FRI_ROUNDS + 16], sizeof(fin));
  if (!ef_eq(fin[0], fin[1]) && !(shard && shard->solo))
    throw std::runtime_error("FRI: final polynomial is not constant (trace violates the AIR)");
  const uint32_t witness = tbox[T_RES];
  if (tbox[T_RES + 1] != 1) throw std::runtime_error("grind: bad witness");
  {  // The host replays the device's FRI transcript (fri::prover: observe each commit-phase
     // root, sample its beta; observe the final constant; the witness check; the query indices)
     // and must arrive at the device's challenger and the device's query indices.
    for (int i = 0; i < nt; i++) {
      ch.observe_digest(trees[i].root);
      (void)ch.sample_ef();
    }
    ch.observe_ef(fin[0]);
    if (!ch.check_witness(POW_BITS, witness))
      throw std::runtime_error("device transcript diverged from the host challenger: PoW witness");
    for (int q = 0; q < nq; q++)
      if (ch.sample_bits(Lmax) != tbox[T_Q + q])
        throw std::runtime_error("device transcript diverged from the host challenger: query index");
    DevChallenger dc;
    std::memcpy(&dc, &tbox[T_CH], sizeof(dc));
    if (std::memcmp(ch.st, dc.st, 64) != 0 || ch.nin != (int)dc.nin || ch.nout != (int)dc.nout ||
        std::memcmp(ch.in, dc.in, 4 * (size_t)ch.nin) != 0 ||
        std::memcmp(ch.out, dc.out, 4 * (size_t)ch.nout) != 0)
      throw std::runtime_error("device transcript diverged from the host challenger: final state");
  }
  if (after) *after = ch;  // the transcript is complete: MachineProver::open's &mut challenger
  const uint32_t* words = tbox + T_W;
  if (ev.on) ev.end(e4, st, &tms->fri);
  span.end();

  // ---- serialize (BFZ1 normal form)
  Writer w;
  w.reserve(4 * nwords + ((size_t)64 << 10));
  w.u32(0x315a4642u);
  w.u32((uint32_t)nc);
  for (int k = 0; k < nc; k++) {
    const char* nm = CHIP_INFO[chip[k]].name;
    w.u32((uint32_t)chip[k]);
    w.u32((uint32_t)std::strlen(nm));
    w.bytes(nm, std::strlen(nm));
  }
  w.digest(mainr.tree.root);
  w.digest(permr.tree.root);
  w.digest(quotr.tree.root);
  auto write_vals = [&](size_t off, int n) {
    w.u32((uint32_t)n);
    for (int c = 0; c < n; c++) w.ef(opened[off + c]);
  };
  for (int k = 0; k < nc; k++) {
    w.u32((uint32_t)mainr.mats[k].log_n);
    const int pi = pk.idx_of_chip[chip[k]];
    if (pi >= 0) {
      const int pw = pk.prep.mats[pi].lde.width;
      write_vals(mp[0][pi].off[0], pw);
      write_vals(mp[0][pi].off[1], pw);
    } else {
      w.u32(0);
      w.u32(0);
    }
    const int mw = mainr.mats[k].lde.width;
    write_vals(mp[1][k].off[0], mw);
    if (mp[1][k].npts == 2) {
      write_vals(mp[1][k].off[1], mw);
    } else {
      w.u32((uint32_t)mw);
      for (int c = 0; c < mw; c++) w.ef(ef_zero());
    }
    const int pw = permr.mats[k].lde.width;
    write_vals(mp[2][k].off[0], pw);
    write_vals(mp[2][k].off[1], pw);
    w.u32(2);
    write_vals(mp[3][2 * k].off[0], 4);
    write_vals(mp[3][2 * k + 1].off[0], 4);
    w.ef(cums[k]);
  }
  w.u32((uint32_t)ncommit);
  for (int i = 0; i < ncommit; i++) w.digest(trees[i].root);
  w.u32((uint32_t)nq);
  w.raw(words, nwords);  // every query in serialized form (canonical words + length words)
  w.ef(fin[0]);
  w.u32(witness);
  htrace().mark("serialized");
  return w.take();
}
}  // namespace

std::vector<uint8_t> prove_events(const ProvingKey& pk, const DeviceEvents& ev,
                                  const ProveOptions& opt, StageTimes* times) {
  hipStream_t st = stream();
  const bool timing = opt.timing && times;
  hipEvent_t a = nullptr, b = nullptr;
  if (timing) {
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    HIP_CHECK(hipEventRecord(a, st));
  }
  htrace().mark("proof start", true);
  static const bool pool_diag = std::getenv("BFZ_HOST_TRACE") != nullptr;
  const uint64_t m0 = lane().pool.mallocs();
  const double t0 = lane().pool.malloc_ms();
  Span span("prove_shard");  // prover.rs:575
  DeviceTraces dt;
  {
    Span gen("generate traces for shard");  // prover.rs:63
    generate_traces_device(ev, dt, st);
  }
  htrace().mark("traces launched");
  if (timing) HIP_CHECK(hipEventRecord(b, st));
  auto proof = prove_device(pk, dt, opt, times);
  htrace().mark("proof returned");
  if (pool_diag)  // the proof's hipMalloc calls (a first proof fills the lane's pool)
    std::fprintf(stderr, "pool: %llu hipMalloc in this proof, %.3f ms of host time\n",
                 (unsigned long long)(lane().pool.mallocs() - m0), lane().pool.malloc_ms() - t0);
  if (timing) {
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    times->trace = ms;
    times->total += ms;
    HIP_CHECK(hipEventDestroy(a));
    HIP_CHECK(hipEventDestroy(b));
  }
  return proof;
}

std::vector<uint8_t> prove(const ProvingKey& pk, const uint8_t* in, size_t nin,
                           const ProveOptions& opt, StageTimes* times,
                           std::vector<uint8_t>* output_stream, uint64_t* cycles) {
  HostEvents& h = scratch_events();  // the pipeline executor into pinned memory
  execute_into(pk.program, in, nin, h);
  DeviceEvents ev;
  upload_events(h, pk.program, ev, stream());
  if (output_stream) *output_stream = h.output;
  if (cycles) *cycles = h.global_clk;
  return prove_events(pk, ev, opt, times);
}

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_prover{(const void*)&k_pack_fri_tail};

}  // namespace bfz
