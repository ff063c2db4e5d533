// Host verifier (see verifier.h).  Checks, in the reference's order:
//   BfProver::verify           (crates/prover/src/verify.rs:10-36): Cpu present, log deg <= 22
//   Verifier::verify_shard     (crates/stark/src/verifier.rs:27-216): byte-multiplicity bound,
//                              transcript replay, PCS/FRI verification, per-chip OOD check
//                              folded(zeta) * 1/Z_H(zeta) == recomputed quotient(zeta),
//                              sum of cumulative sums == 0.
#include "verifier.h"
#include "host_p2.h"

#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <stdexcept>
#include <vector>

#include "air.h"
#include "machine.h"
#include "poseidon2.h"
#include "prover.h"

namespace bfz {

using namespace kb;

namespace {

constexpr int LOG_BLOWUP = 1, POW_BITS = 16, MAX_CPU_LOG_DEGREE = 22;

struct HornerAcc {
  EF acc = ef_zero();
  EF alpha;
  void emit(const EF& c) { acc = ef_add(ef_mul(acc, alpha), c); }
  void emit_ext(const EF& c) { emit(c); }
};

template <int CHIP>
EF fold_chip(const std::vector<EF>& pl, const std::vector<EF>& pn, const std::vector<EF>& ml,
             const std::vector<EF>& mn, const std::vector<EF>& perml, const std::vector<EF>& permn,
             const EF& pa, const EF* pb_pows, const EF& cumsum, const EF& first, const EF& last,
             const EF& trans, const EF& alpha) {
  HornerAcc acc;
  acc.alpha = alpha;
  static const EF zero1[1] = {ef_zero()};
  const EF* PL = pl.empty() ? zero1 : pl.data();
  const EF* PN = pn.empty() ? zero1 : pn.data();
  Air<ExtOps, HornerAcc> air{ml.data(), mn.data(), PL, PN, first, last, trans, acc};
  air.template eval_air<CHIP>();
  air.template eval_perm<CHIP>(perml.data(), permn.data(), pa, pb_pows, cumsum, first, last, trans);
  return acc.acc;
}

EF fold_any(int chip, const std::vector<EF>& pl, const std::vector<EF>& pn, const std::vector<EF>& ml,
            const std::vector<EF>& mn, const std::vector<EF>& perml, const std::vector<EF>& permn,
            const EF& pa, const EF* pb, const EF& cs, const EF& f, const EF& l, const EF& t,
            const EF& al) {
  switch (chip) {
    case CHIP_CPU: return fold_chip<CHIP_CPU>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_PROGRAM: return fold_chip<CHIP_PROGRAM>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_ADDSUB: return fold_chip<CHIP_ADDSUB>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_JUMP: return fold_chip<CHIP_JUMP>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_MEMORY: return fold_chip<CHIP_MEMORY>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_BYTE: return fold_chip<CHIP_BYTE>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_MEMINSTRS: return fold_chip<CHIP_MEMINSTRS>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
    case CHIP_IO: return fold_chip<CHIP_IO>(pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al);
  }
  throw std::runtime_error("bad chip");
}

void sponge(uint32_t st[16], const std::vector<const uint32_t*>& rows, const std::vector<int>& ws) {
  int pos = 0;
  for (size_t m = 0; m < rows.size(); m++)
    for (int c = 0; c < ws[m]; c++) {
      st[pos++] = rows[m][c];
      if (pos == 8) {
        host_permute(st);
        pos = 0;
      }
    }
  if (pos) host_permute(st);
}

void compress(const uint32_t* l, const uint32_t* r, uint32_t* out) {
  uint32_t s[16];
  std::memcpy(s, l, 32);
  std::memcpy(s + 8, r, 32);
  host_permute(s);
  std::memcpy(out, s, 32);
}

// MerkleTreeMmcs::verify_batch [p3-recalled]; heights are powers of two.
bool verify_batch(const uint32_t root[8], const std::vector<size_t>& heights,
                  const std::vector<int>& widths, size_t index,
                  const std::vector<std::vector<uint32_t>>& rows,
                  const std::vector<uint32_t>& path) {
  std::vector<int> ord(heights.size());
  for (size_t i = 0; i < ord.size(); i++) ord[i] = (int)i;
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return heights[a] > heights[b]; });
  size_t cur = heights[ord[0]];
  size_t k = 0;
  auto take = [&](std::vector<const uint32_t*>& rp, std::vector<int>& wp) {
    while (k < ord.size() && heights[ord[k]] == cur) {
      rp.push_back(rows[ord[k]].data());
      wp.push_back(widths[ord[k]]);
      k++;
    }
  };
  std::vector<const uint32_t*> rp;
  std::vector<int> wp;
  take(rp, wp);
  uint32_t h[16] = {0};
  sponge(h, rp, wp);
  uint32_t node[8];
  std::memcpy(node, h, 32);
  for (size_t L = 0; L < path.size() / 8; L++) {
    const uint32_t* sib = &path[8 * L];
    if (index & 1) compress(sib, node, node);
    else compress(node, sib, node);
    index >>= 1;
    cur >>= 1;
    if (k < ord.size() && heights[ord[k]] == cur) {
      rp.clear();
      wp.clear();
      take(rp, wp);
      uint32_t hh[16] = {0};
      sponge(hh, rp, wp);
      compress(node, hh, node);
    }
  }
  return k == ord.size() && std::memcmp(node, root, 32) == 0;
}

EF monomial(int e) {
  EF m = ef_zero();
  m.c[e] = ONE;
  return m;
}

EF zp_at(int log_n, uint32_t shift, const EF& x) {  // (x / s)^(2^log_n) - 1
  EF u = ef_mul_base(x, minv(shift));
  for (int i = 0; i < log_n; i++) u = ef_mul(u, u);
  return ef_sub(u, ef_one());
}

// number of byte lookups each chip SENDS (Chip::num_sent_byte_lookups)
int sent_byte_lookups(int chip) { return chip == CHIP_CPU ? 7 : chip == CHIP_ADDSUB ? 3 : 0; }

}  // namespace

bool verify_proof(const std::string& src, const uint32_t vk_commit[8], const uint8_t* proof,
                  size_t len, const VerifyOptions& opt, std::string* why) {
  ShardProof pf;
  try {
    pf = decode_bfz1(proof, len);
  } catch (const std::exception& e) {
    if (why) *why = e.what();
    return false;
  }
  return verify_shard(src, vk_commit, pf, opt, why);
}

bool verify_shard(const std::string& src, const uint32_t vk_commit[8], const ShardProof& pf,
                  const VerifyOptions& opt, std::string* why) {
  try {
    Program prog = Program::parse(src);
    // vk.chip_information: prep matrices sorted by (Reverse(height), name)
    size_t prog_h = std::max<size_t>(16, [&] {
      size_t p = 1;
      while (p < prog.instructions.size()) p <<= 1;
      return p;
    }());
    struct PrepInfo { int chip; int log_n; int w; };
    std::vector<PrepInfo> prep = {{CHIP_PROGRAM, log2i(prog_h), 6}, {CHIP_BYTE, 16, 2}};
    if (prep[1].log_n > prep[0].log_n ||
        (prep[1].log_n == prep[0].log_n && std::strcmp("Byte", "Program") < 0))
      std::swap(prep[0], prep[1]);

    const uint32_t nc = (uint32_t)pf.chips.size();
    if (nc == 0 || nc > NUM_CHIPS || pf.opened.size() != nc) throw std::runtime_error("bad chip count");
    const std::vector<int>& chip = pf.chips;
    {
      std::vector<bool> seen(NUM_CHIPS, false);
      for (int c : chip) {
        if (c < 0 || c >= NUM_CHIPS || seen[c]) throw std::runtime_error("bad chip id");
        seen[c] = true;
      }
    }
    const uint32_t* main_root = pf.main_root.data();
    const uint32_t* perm_root = pf.perm_root.data();
    const uint32_t* quot_root = pf.quot_root.data();
    struct ChipOpen {
      int log_n;
      const std::vector<EF> &pl, &pn, &ml, &mn, &perml, &permn;
      const std::vector<EF>* q;
      EF cumsum;
    };
    std::vector<ChipOpen> co;
    co.reserve(nc);
    for (uint32_t i = 0; i < nc; i++) {
      const ChipOpened& o = pf.opened[i];
      // unsigned: a huge word must not become a negative shift count below
      // log degree 0 is a 1-row trace (the Cpu chip of a one-cycle program: cpu/trace.rs:33
      // pads to next_power_of_two with no minimum)
      if (o.log_degree > 23) throw std::runtime_error("log degree out of range");
      co.push_back(ChipOpen{(int)o.log_degree, o.prep_local, o.prep_next, o.main_local, o.main_next,
                            o.perm_local, o.perm_next, o.quotient, o.cumsum});
      const ChipOpen& c = co.back();
      const int ch = chip[i];
      const size_t pw = CHIP_INFO[ch].prep_w;
      if (c.ml.size() != (size_t)CHIP_INFO[ch].main_w || c.mn.size() != c.ml.size() ||
          c.perml.size() != 4 * (size_t)perm_width(ch) || c.permn.size() != c.perml.size() ||
          c.pl.size() != pw || c.pn.size() != pw || c.q[0].size() != 4 || c.q[1].size() != 4)
        throw std::runtime_error("opened-value shape mismatch");
      // A local-only chip's next values are not opened by the PCS (verifier.rs:109-135), so
      // the reference verifier would accept any words there; its prover writes zeros
      // (prover.rs:484-487, 499-502).  Requiring the zeros keeps accepted proofs
      // non-malleable (tests/test_abi.py fuzz) and rejects nothing an honest prover emits.
      if (CHIP_INFO[ch].local_only) {
        for (const std::vector<EF>* v : {&c.pn, &c.mn})
          for (const EF& e : *v)
            if (e.c[0] | e.c[1] | e.c[2] | e.c[3])
              throw std::runtime_error("local-only chip with non-zero next values");
      }
    }
    // BfProver::verify: Cpu chip present, log degree bound
    int cpu_i = -1;
    for (uint32_t i = 0; i < nc; i++) if (chip[i] == CHIP_CPU) cpu_i = (int)i;
    if (cpu_i < 0) throw std::runtime_error("missing Cpu chip");
    if (co[cpu_i].log_n > MAX_CPU_LOG_DEGREE) throw std::runtime_error("Cpu log degree too large");
    // byte multiplicities must not overflow (verifier.rs:47-62)
    {
      unsigned __int128 tot = 0;
      for (uint32_t i = 0; i < nc; i++) tot += (unsigned __int128)sent_byte_lookups(chip[i]) << co[i].log_n;
      if (tot > P) throw std::runtime_error("byte multiplicities overflow");
    }
    // ---- transcript (verifier.rs:76-101)
    Challenger ch;
    ch.observe_digest(vk_commit);
    for (int i = 0; i < 7; i++) ch.observe(0);
    ch.observe_digest(main_root);
    const EF pa = ch.sample_ef(), pb = ch.sample_ef();
    ch.observe_digest(perm_root);
    for (uint32_t i = 0; i < nc; i++) {
      ch.observe_ef(co[i].cumsum);
      // chips with no interactions must have a zero sum (all chips here have interactions)
    }
    const EF alpha = ch.sample_ef();
    ch.observe_digest(quot_root);
    const EF zeta = ch.sample_ef();

    // ---- rounds for PCS verify
    struct VMat { int log_n; uint32_t shift; int w; int np; EF pt[2]; const std::vector<EF>* v[2]; };
    std::vector<VMat> rounds[4];
    for (const PrepInfo& pi : prep) {
      int idx = -1;
      for (uint32_t j = 0; j < nc; j++) if (chip[j] == pi.chip) idx = (int)j;
      if (idx < 0) throw std::runtime_error("preprocessed chip missing from proof");
      VMat m{pi.log_n, ONE, pi.w, CHIP_INFO[pi.chip].local_only ? 1 : 2, {zeta, ef_mul_base(zeta, two_adic_gen(pi.log_n))},
             {&co[idx].pl, &co[idx].pn}};
      rounds[0].push_back(m);
    }
    for (uint32_t i = 0; i < nc; i++) {
      const ChipOpen& c = co[i];
      const EF znext = ef_mul_base(zeta, two_adic_gen(c.log_n));
      rounds[1].push_back(VMat{c.log_n, ONE, (int)c.ml.size(), CHIP_INFO[chip[i]].local_only ? 1 : 2,
                               {zeta, znext}, {&c.ml, &c.mn}});
      rounds[2].push_back(VMat{c.log_n, ONE, (int)c.perml.size(), 2, {zeta, znext}, {&c.perml, &c.permn}});
      const uint32_t w2n = two_adic_gen(c.log_n + 1);
      for (int k = 0; k < 2; k++)
        rounds[3].push_back(VMat{c.log_n, mmul(to_mont(3), k ? w2n : ONE), 4, 1, {zeta, zeta},
                                 {&c.q[k], &c.q[k]}});
    }
    if (opt.observe_openings)  // decision D1: opened values enter the transcript
      for (int rr = 0; rr < 4; rr++)
        for (const VMat& m : rounds[rr])
          for (int p = 0; p < m.np; p++)
            for (int c = 0; c < m.w; c++) ch.observe_ef((*m.v[p])[c]);
    const EF fri_alpha = ch.sample_ef();
    const uint32_t ncommit = (uint32_t)pf.commit_roots.size();
    if (ncommit > 30) throw std::runtime_error("too many FRI rounds");
    const int log_max = (int)ncommit + LOG_BLOWUP;
    {  // the commit phase folds the tallest LDE down to 2^LOG_BLOWUP: every height must fit
      int lh_max = 0;
      for (int rr = 0; rr < 4; rr++)
        for (const VMat& m : rounds[rr]) lh_max = std::max(lh_max, m.log_n + LOG_BLOWUP);
      if (lh_max != log_max) throw std::runtime_error("FRI round count does not match the tallest matrix");
    }
    std::vector<EF> betas(ncommit);
    for (uint32_t i = 0; i < ncommit; i++) {
      ch.observe_digest(pf.commit_roots[i].data());
      betas[i] = ch.sample_ef();
    }
    const uint32_t nq = (uint32_t)pf.queries.size();
    if ((int)nq != opt.num_queries) throw std::runtime_error("wrong number of queries");
    const EF final_poly = pf.final_poly;
    ch.observe_ef(final_poly);
    if (!ch.check_witness(POW_BITS, from_mont(pf.pow_witness))) throw std::runtime_error("bad PoW witness");
    const uint32_t* roots[4] = {vk_commit, main_root, perm_root, quot_root};
    const uint32_t half = to_mont_c((P + 1) / 2);
    (void)half;
    for (uint32_t q = 0; q < nq; q++) {
      const QueryProof& qp = pf.queries[q];
      const size_t index = ch.sample_bits(log_max);
      if (qp.inputs.size() != 4) throw std::runtime_error("bad round count");
      std::map<int, std::pair<EF, EF>> ro;  // log height -> (alpha_pow, ro)
      for (int rr = 0; rr < 4; rr++) {
        const BatchOpening& bo = qp.inputs[rr];
        const size_t nm = bo.rows.size();
        if (nm != rounds[rr].size()) throw std::runtime_error("bad matrix count");
        const std::vector<std::vector<uint32_t>>& rows = bo.rows;
        std::vector<size_t> heights(nm);
        std::vector<int> widths(nm);
        int lbmax = 0;
        for (size_t i = 0; i < nm; i++) {
          const size_t w = rows[i].size();
          if ((int)w != rounds[rr][i].w) throw std::runtime_error("bad row width");
          heights[i] = (size_t)1 << (rounds[rr][i].log_n + LOG_BLOWUP);
          widths[i] = (int)w;
          lbmax = std::max(lbmax, rounds[rr][i].log_n + LOG_BLOWUP);
        }
        if ((int)bo.path.size() != lbmax) throw std::runtime_error("bad path length");
        std::vector<uint32_t> path(8 * bo.path.size());
        for (size_t L = 0; L < bo.path.size(); L++) std::memcpy(&path[8 * L], bo.path[L].data(), 32);
        const size_t ridx = index >> (log_max - lbmax);
        if (!verify_batch(roots[rr], heights, widths, ridx, rows, path))
          throw std::runtime_error("input Merkle opening rejected");
        for (uint32_t i = 0; i < nm; i++) {
          const VMat& m = rounds[rr][i];
          const int lh = m.log_n + LOG_BLOWUP;
          const uint32_t rev = bitrev32((uint32_t)(index >> (log_max - lh)), lh);
          const uint32_t x = mmul(to_mont(3), mpow(two_adic_gen(lh), rev));
          auto it = ro.find(lh);
          if (it == ro.end()) it = ro.emplace(lh, std::make_pair(ef_one(), ef_zero())).first;
          for (int p = 0; p < m.np; p++) {
            const EF inv = ef_inv(ef_sub(ef_base(x), m.pt[p]));
            for (int c = 0; c < m.w; c++) {
              const EF quo = ef_mul(ef_sub(ef_base(rows[i][c]), (*m.v[p])[c]), inv);
              it->second.second = ef_add(it->second.second, ef_mul(it->second.first, quo));
              it->second.first = ef_mul(it->second.first, fri_alpha);
            }
          }
        }
      }
      // verify_query
      if (qp.steps.size() != ncommit) throw std::runtime_error("bad step count");
      EF folded = ef_zero();
      size_t idx = index;
      for (uint32_t s = 0; s < ncommit; s++) {
        const int lfh = log_max - 1 - (int)s;
        auto it = ro.find(lfh + 1);
        if (it != ro.end()) {
          folded = ef_add(folded, it->second.second);
          ro.erase(it);
        }
        const CommitPhaseStep& stp = qp.steps[s];
        const EF sib = stp.sibling;
        if ((int)stp.path.size() != lfh) throw std::runtime_error("bad FRI path length");
        std::vector<uint32_t> path(8 * stp.path.size());
        for (size_t L = 0; L < stp.path.size(); L++) std::memcpy(&path[8 * L], stp.path[L].data(), 32);
        EF ev[2];
        ev[idx & 1] = folded;
        ev[(idx & 1) ^ 1] = sib;
        std::vector<std::vector<uint32_t>> row(1, std::vector<uint32_t>(8));
        std::memcpy(row[0].data(), ev[0].c, 16);
        std::memcpy(row[0].data() + 4, ev[1].c, 16);
        if (!verify_batch(pf.commit_roots[s].data(), {(size_t)1 << lfh}, {8}, idx >> 1, row, path))
          throw std::runtime_error("FRI commit-phase opening rejected");
        idx >>= 1;
        const uint32_t x0 = mpow(two_adic_gen(lfh + 1), bitrev32((uint32_t)idx, lfh));
        const uint32_t x1 = mneg(x0);
        const EF t = ef_mul(ef_sub(betas[s], ef_base(x0)), ef_sub(ev[1], ev[0]));
        folded = ef_add(ev[0], ef_mul_base(t, minv(msub(x1, x0))));
      }
      {  // a 1-row trace's height-2 input joins after the last fold, as in the commit phase (D11)
        auto it = ro.find(log_max - (int)ncommit);
        if (it != ro.end()) {
          folded = ef_add(folded, it->second.second);
          ro.erase(it);
        }
      }
      if (!ro.empty()) throw std::runtime_error("unconsumed reduced openings");
      if (!ef_eq(folded, final_poly)) throw std::runtime_error("FRI final value mismatch");
    }

    // ---- OOD constraint checks (verifier.rs:194-213)
    EF total = ef_zero();
    for (uint32_t i = 0; i < nc; i++) {
      const ChipOpen& c = co[i];
      const int n_log = c.log_n;
      const uint32_t w2n = two_adic_gen(n_log + 1);
      const uint32_t sh[2] = {to_mont(3), mmul(to_mont(3), w2n)};
      EF zps[2];
      for (int a = 0; a < 2; a++) {
        const int o = 1 - a;
        zps[a] = ef_mul(zp_at(n_log, sh[o], zeta), ef_inv(zp_at(n_log, sh[o], ef_base(sh[a]))));
      }
      EF quot = ef_zero();
      for (int a = 0; a < 2; a++)
        for (int e = 0; e < 4; e++) quot = ef_add(quot, ef_mul(ef_mul(zps[a], monomial(e)), c.q[a][e]));
      const uint32_t gn_inv = minv(two_adic_gen(n_log));
      EF zh = zeta;
      for (int k = 0; k < n_log; k++) zh = ef_mul(zh, zh);
      zh = ef_sub(zh, ef_one());
      const EF first = ef_mul(zh, ef_inv(ef_sub(zeta, ef_one())));
      const EF last = ef_mul(zh, ef_inv(ef_sub(zeta, ef_base(gn_inv))));
      const EF trans = ef_sub(zeta, ef_base(gn_inv));
      const int pw = perm_width(chip[i]);
      std::vector<EF> perml(pw), permn(pw);
      for (int e = 0; e < pw; e++) {
        perml[e] = ef_zero();
        permn[e] = ef_zero();
        for (int k = 0; k < 4; k++) {
          perml[e] = ef_add(perml[e], ef_mul(monomial(k), c.perml[4 * e + k]));
          permn[e] = ef_add(permn[e], ef_mul(monomial(k), c.permn[4 * e + k]));
        }
      }
      EF pb_pows[8];
      pb_pows[0] = ef_one();
      for (int j = 1; j < 8; j++) pb_pows[j] = ef_mul(pb_pows[j - 1], pb);
      const EF folded = fold_any(chip[i], c.pl, c.pn, c.ml, c.mn, perml, permn, pa, pb_pows, c.cumsum,
                                 first, last, trans, alpha);
      if (!ef_eq(ef_mul(folded, ef_inv(zh)), quot))
        throw std::runtime_error(std::string("OOD evaluation mismatch on chip ") + CHIP_INFO[chip[i]].name);
      total = ef_add(total, c.cumsum);
    }
    if (!ef_is_zero(total)) throw std::runtime_error("cumulative sums do not sum to zero");
    return true;
  } catch (const std::exception& e) {
    if (why) *why = e.what();
    return false;
  }
}

// Columns a chip's constraints read at the next row (quotient.rs:41-42), found by perturbing
// one next-row value at a time in a random evaluation of fold_any (a column the constraints do
// not read cannot change the folded value; one that they read changes it except with
// probability ~1/p).  The sharded prover computes next-row shards only for these columns.
NextCols next_row_columns(int chip) {
  const ChipInfo& ci = CHIP_INFO[chip];
  uint64_t seed = 0x9E3779B97F4A7C15ull * (uint64_t)(chip + 1);
  auto rnd = [&] {
    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
    return to_mont((uint32_t)((seed >> 33) % P));
  };
  auto rnd_ef = [&] { return EF{{rnd(), rnd(), rnd(), rnd()}}; };
  auto vec = [&](size_t n) {
    std::vector<EF> v(n);
    for (EF& e : v) e = rnd_ef();
    return v;
  };
  const size_t pw = (size_t)perm_width(chip);  // fold_any takes the perm values as EF columns
  std::vector<EF> pl = vec(ci.prep_w), pn = vec(ci.prep_w), ml = vec(ci.main_w), mn = vec(ci.main_w),
                  perml = vec(pw), permn = vec(pw);
  EF pb[8];
  for (EF& e : pb) e = rnd_ef();
  const EF pa = rnd_ef(), cs = rnd_ef(), f = rnd_ef(), l = rnd_ef(), t = rnd_ef(), al = rnd_ef();
  auto fold = [&] { return fold_any(chip, pl, pn, ml, mn, perml, permn, pa, pb, cs, f, l, t, al); };
  const EF base = fold();
  NextCols nc;
  for (int pass = 0; pass < 2; pass++) {
    std::vector<EF>& v = pass ? permn : mn;
    for (size_t c = 0; c < v.size(); c++) {
      const EF keep = v[c];
      v[c] = ef_add(v[c], ef_one());
      if (!ef_eq(fold(), base)) {
        if (pass)
          for (int k = 0; k < 4; k++) nc.perm.push_back(4 * (int)c + k);  // flatten_to_base
        else
          nc.main.push_back((int)c);
      }
      v[c] = keep;
    }
  }
  return nc;
}

}  // namespace bfz
