// AIR constraints and LogUp interactions of the 8 Brainfuck chips, written once as templates
// over an arithmetic "Ops" policy:
//   - BaseOps: trace values in the base field (GPU quotient kernel, prover side);
//   - ExtOps : trace values in the extension (host verifier, OOD evaluation at zeta).
// Constraint ORDER matters (acc = acc*alpha + c, crates/stark/src/folder.rs:68-72); each
// function cites the reference eval it follows.  Chip::eval evaluates the AIR first and the
// LogUp constraints after (crates/stark/src/chip.rs:222-228).
#pragma once
#include <type_traits>

#include "kb.h"

namespace bfz {

using kb::EF;

// ------------------------------------------------------------------- arithmetic policies
struct BaseOps {
  using T = uint32_t;
  static KB_HD T add(T a, T b) { return kb::madd(a, b); }
  static KB_HD T sub(T a, T b) { return kb::msub(a, b); }
  static KB_HD T mul(T a, T b) { return kb::mmul(a, b); }
  static KB_HD T neg(T a) { return kb::mneg(a); }
  static KB_HD T cst(uint32_t mont) { return mont; }
  static KB_HD EF toE(T a) { return kb::ef_base(a); }
  static KB_HD EF mulE(const EF& e, T a) { return kb::ef_mul_base(e, a); }
};
struct ExtOps {
  using T = EF;
  static KB_HD T add(const T& a, const T& b) { return kb::ef_add(a, b); }
  static KB_HD T sub(const T& a, const T& b) { return kb::ef_sub(a, b); }
  static KB_HD T mul(const T& a, const T& b) { return kb::ef_mul(a, b); }
  static KB_HD T neg(const T& a) { return kb::ef_neg(a); }
  static KB_HD T cst(uint32_t mont) { return kb::ef_base(mont); }
  static KB_HD EF toE(const T& a) { return a; }
  static KB_HD EF mulE(const EF& e, const T& a) { return kb::ef_mul(e, a); }
};

constexpr uint32_t MC(uint32_t x) { return kb::to_mont_c(x); }

// ------------------------------------------------------------------- LogUp interactions
// LookupKind argument indices (crates/stark/src/lookup/lookup.rs:17-42)
enum : uint8_t { K_MEMORY = 1, K_PROGRAM = 2, K_ALU = 3, K_JUMP = 4, K_MEMINSTR = 5, K_IO = 6, K_BYTE = 7 };
enum : uint8_t { S_MAIN = 0, S_PREP = 1 };

struct VTerm { uint8_t src, col; uint32_t w; };  // weight: canonical small integer
struct VCol {                                   // VirtualPairCol: c + sum w_i * col_i
  uint8_t n;
  VTerm t[4];
  uint32_t c;
};
struct Lookup {
  uint8_t kind, nvals;
  bool send;
  VCol vals[7];
  VCol mult;
};
struct ChipLookups {
  int n;
  Lookup l[16];  // chain order: sends (emission order) then receives (emission order)
};

constexpr VCol vc(uint32_t c) { return VCol{0, {}, c}; }
constexpr VCol vm(uint8_t col) { return VCol{1, {{S_MAIN, col, 1}}, 0}; }
constexpr VCol vp(uint8_t col) { return VCol{1, {{S_PREP, col, 1}}, 0}; }
constexpr VCol vm2(uint8_t a, uint32_t wa, uint8_t b, uint32_t wb, uint32_t c = 0) {
  return VCol{2, {{S_MAIN, a, wa}, {S_MAIN, b, wb}}, c};
}
constexpr VCol vword(uint8_t col) {  // Word::reduce (crates/stark/src/word.rs:66-70)
  return VCol{4, {{S_MAIN, col, 1}, {S_MAIN, (uint8_t)(col + 1), 1u << 8},
                  {S_MAIN, (uint8_t)(col + 2), 1u << 16}, {S_MAIN, (uint8_t)(col + 3), 1u << 24}}, 0};
}

// Cpu: cpu/air.rs:28-98 -> air/program.rs:12-27, air/memory.rs:17-125, air/u8_air.rs:7-15.
// clk = clk_16 + 2^16 clk_8 (cols 0,1).
constexpr ChipLookups CPU_LOOKUPS = {16, {
  {K_PROGRAM, 7, true, {vm(2), vm(8), vm(8), vm(9), vm(10), vm(11), vm(12)}, vm(30)},
  {K_ALU, 4, true, {vm(2), vm(8), vm(7), vm(6)}, vm(26)},
  {K_JUMP, 4, true, {vm(2), vm(3), vm(8), vm(6)}, vm(27)},
  {K_MEMINSTR, 5, true, {vm2(0, 1, 1, 1u << 16), vm(2), vm(8), vm(4), vm(5)}, vm(29)},
  {K_IO, 4, true, {vm(2), vm(8), vm(4), vm(6)}, vm(28)},
  {K_BYTE, 3, true, {vc(1), vc(0), vm(16)}, vm(23)},       // mv_access diff 16-bit limb
  {K_BYTE, 3, true, {vc(0), vm(17), vc(0)}, vm(23)},       // mv_access diff 8-bit limb
  {K_MEMORY, 3, true, {vm(15), vm(4), vm(13)}, vm(23)},    // (prev_clk, mp, prev_value)
  {K_BYTE, 3, true, {vc(1), vc(0), vm(21)}, vm(24)},       // next_mv_access limbs
  {K_BYTE, 3, true, {vc(0), vm(22), vc(0)}, vm(24)},
  {K_MEMORY, 3, true, {vm(20), vm(4), vm(18)}, vm(24)},
  {K_BYTE, 3, true, {vc(0), vm(6), vc(0)}, vm(30)},        // range_check_u8(mv)
  {K_BYTE, 3, true, {vc(1), vc(0), vm(0)}, vm(30)},        // clk 16-bit limb
  {K_BYTE, 3, true, {vc(0), vm(1), vc(0)}, vm(30)},        // clk 8-bit limb
  {K_MEMORY, 3, false, {vm2(0, 1, 1, 1u << 16, 1), vm(4), vm(14)}, vm(23)},  // (clk+1, mp, value)
  {K_MEMORY, 3, false, {vm2(0, 1, 1, 1u << 16, 2), vm(4), vm(19)}, vm(24)},  // (clk+2, ...)
}};
// Program: program/mod.rs:152-163 (receive_program: pc, opcode, opcode, op_a[0..4])
constexpr ChipLookups PROGRAM_LOOKUPS = {1, {
  {K_PROGRAM, 7, false, {vp(0), vp(1), vp(1), vp(2), vp(3), vp(4), vp(5)}, vm(0)},
}};
// AddSub: alu/mod.rs:155-193, operations/add.rs:44-76
constexpr ChipLookups ADDSUB_LOOKUPS = {5, {
  {K_BYTE, 3, true, {vc(0), vm(3), vc(0)}, vm2(5, 1, 6, 1)},
  {K_BYTE, 3, true, {vc(0), vm(4), vc(0)}, vm2(5, 1, 6, 1)},
  {K_BYTE, 3, true, {vc(0), vm(1), vc(0)}, vm2(5, 1, 6, 1)},
  {K_ALU, 4, false, {vm(0), vc(2), vm(1), vm(3)}, vm(5)},
  {K_ALU, 4, false, {vm(0), vc(3), vm(3), vm(1)}, vm(6)},
}};
// Jump: jump/air.rs:72-81
constexpr ChipLookups JUMP_LOOKUPS = {1, {
  {K_JUMP, 4, false, {vword(0), vword(18), vm2(43, 0, 44, 1), vm(40)}, vm2(43, 1, 44, 1)},
}};
// Memory: memory/memory.rs:132-145 (per entry: receive initial, send final)
constexpr ChipLookups MEMORY_LOOKUPS = {4, {
  {K_MEMORY, 3, true, {vm(2), vm(0), vm(4)}, vm(5)},
  {K_MEMORY, 3, true, {vm(8), vm(6), vm(10)}, vm(11)},
  {K_MEMORY, 3, false, {vm(1), vm(0), vm(3)}, vm(5)},
  {K_MEMORY, 3, false, {vm(7), vm(6), vm(9)}, vm(11)},
}};
// Byte: bytes/air.rs:21-44
constexpr ChipLookups BYTE_LOOKUPS = {2, {
  {K_BYTE, 3, false, {vc(0), vp(0), vc(0)}, vm(0)},
  {K_BYTE, 3, false, {vc(1), vc(0), vp(1)}, vm(1)},
}};
// MemoryInstrs: memory/instructions/air.rs:65-75
constexpr ChipLookups MEMINSTRS_LOOKUPS = {1, {
  {K_MEMINSTR, 5, false, {vm(1), vm(0), vm2(38, 4, 39, 5), vword(2), vword(20)}, vm2(38, 1, 39, 1)},
}};
// IO: io/mod.rs:127-141
constexpr ChipLookups IO_LOOKUPS = {1, {
  {K_IO, 4, false, {vm(0), vm2(3, 6, 4, 7), vm(1), vm(2)}, vm2(3, 1, 4, 1)},
}};

template <int CHIP> struct LookupsOf;
template <> struct LookupsOf<0> { static constexpr const ChipLookups& v = CPU_LOOKUPS; };
template <> struct LookupsOf<1> { static constexpr const ChipLookups& v = PROGRAM_LOOKUPS; };
template <> struct LookupsOf<2> { static constexpr const ChipLookups& v = ADDSUB_LOOKUPS; };
template <> struct LookupsOf<3> { static constexpr const ChipLookups& v = JUMP_LOOKUPS; };
template <> struct LookupsOf<4> { static constexpr const ChipLookups& v = MEMORY_LOOKUPS; };
template <> struct LookupsOf<5> { static constexpr const ChipLookups& v = BYTE_LOOKUPS; };
template <> struct LookupsOf<6> { static constexpr const ChipLookups& v = MEMINSTRS_LOOKUPS; };
template <> struct LookupsOf<7> { static constexpr const ChipLookups& v = IO_LOOKUPS; };

// Evaluate a VirtualPairCol over a row.
template <class Ops>
KB_HD typename Ops::T vcol_eval(const VCol& v, const typename Ops::T* prep, const typename Ops::T* main) {
  typename Ops::T r = Ops::cst(kb::to_mont(v.c));
#pragma unroll
  for (int i = 0; i < v.n; i++) {
    const typename Ops::T& x = v.t[i].src == S_PREP ? prep[v.t[i].col] : main[v.t[i].col];
    r = Ops::add(r, v.t[i].w == 1 ? x : Ops::mul(Ops::cst(kb::to_mont(v.t[i].w)), x));
  }
  return r;
}

// ------------------------------------------------------------------- constraint helpers
// Accumulators: emit(T) for base-valued constraints, emit_ext(EF) for LogUp constraints.
template <class Ops, class Acc>
struct Air {
  using T = typename Ops::T;
  const T* L;   // main local
  const T* N;   // main next
  const T* PL;  // prep local
  const T* PN;  // prep next
  T first, last, trans;
  Acc& acc;

  KB_HD T add(T a, T b) const { return Ops::add(a, b); }
  KB_HD T sub(T a, T b) const { return Ops::sub(a, b); }
  KB_HD T mul(T a, T b) const { return Ops::mul(a, b); }
  KB_HD T k(uint32_t canon) const { return Ops::cst(kb::to_mont(canon)); }
  KB_HD T boolc(T x) const { return mul(x, sub(x, Ops::cst(kb::ONE))); }  // assert_bool
  KB_HD T one() const { return Ops::cst(kb::ONE); }
  KB_HD T word(const T* w) const {
    T r = w[0];
    r = add(r, mul(w[1], Ops::cst(MC(1u << 8))));
    r = add(r, mul(w[2], Ops::cst(MC(1u << 16))));
    r = add(r, mul(w[3], Ops::cst(MC(1u << 24))));
    return r;
  }

  // KoalaBearWordRangeChecker::range_check (operations/koala_bear_word.rs:47-106)
  KB_HD void word_range_check(const T* v, const T* rc, T is_real) {
    T rec = Ops::cst(0);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      acc.emit(mul(is_real, boolc(rc[i])));
      rec = add(rec, mul(Ops::cst(kb::to_mont(1u << i)), rc[i]));
    }
    acc.emit(mul(is_real, sub(rec, v[3])));
    acc.emit(mul(is_real, rc[7]));
    acc.emit(mul(is_real, sub(rc[8], mul(rc[0], rc[1]))));
    acc.emit(mul(is_real, sub(rc[9], mul(rc[8], rc[2]))));
    acc.emit(mul(is_real, sub(rc[10], mul(rc[9], rc[3]))));
    acc.emit(mul(is_real, sub(rc[11], mul(rc[10], rc[4]))));
    acc.emit(mul(is_real, sub(rc[12], mul(rc[11], rc[5]))));
    acc.emit(mul(is_real, sub(rc[13], mul(rc[12], rc[6]))));
    acc.emit(mul(mul(is_real, rc[13]), add(add(v[0], v[1]), v[2])));
  }

  // CpuChip::eval (cpu/air.rs:28-186)
  KB_HD void eval_cpu() {
    const T c16 = Ops::cst(MC(1u << 16));
    const T clk = add(mul(c16, L[1]), L[0]);
    // eval_registers: eval_memory_access(clk + 1, mp, mv_access, mv_accessed)
    acc.emit(boolc(L[23]));
    acc.emit(mul(L[23], sub(sub(sub(add(clk, k(1)), L[15]), one()), add(L[16], mul(L[17], c16)))));
    // eval_memory_access(clk + 2, mp, next_mv_access, next_mv_accessed)
    acc.emit(boolc(L[24]));
    acc.emit(mul(L[24], sub(sub(sub(add(clk, k(2)), L[20]), one()), add(L[21], mul(L[22], c16)))));
    // when(is_mv_immutable).assert_eq(mv_val, mv_access.prev_value)
    acc.emit(mul(L[25], sub(L[14], L[13])));
    // eval_clk
    acc.emit(mul(first, clk));
    const T next_clk = add(mul(c16, N[1]), N[0]);
    acc.emit(mul(mul(trans, N[30]), sub(add(clk, k(2)), next_clk)));
    acc.emit(mul(L[30], sub(clk, add(L[0], mul(L[1], c16)))));
    // eval_pc
    acc.emit(mul(mul(trans, N[30]), sub(L[3], N[2])));
    acc.emit(mul(mul(mul(trans, L[30]), sub(L[27], one())), sub(L[3], add(L[2], one()))));
    // eval_is_real
    acc.emit(boolc(L[30]));
    acc.emit(mul(first, sub(L[30], one())));
    acc.emit(mul(mul(trans, sub(L[30], one())), N[30]));
    // assert_bool(is_alu, is_jump, is_memory_instr, is_io, is_mv_immutable, mv_accessed,
    //             next_mv_accessed)
    acc.emit(boolc(L[26]));
    acc.emit(boolc(L[27]));
    acc.emit(boolc(L[29]));
    acc.emit(boolc(L[28]));
    acc.emit(boolc(L[25]));
    acc.emit(boolc(L[23]));
    acc.emit(boolc(L[24]));
  }

  // AddSubChip::eval (alu/mod.rs:155-193) + AddOperation::eval (operations/add.rs:44-76)
  KB_HD void eval_addsub() {
    const T is_real = add(L[5], L[6]);
    acc.emit(boolc(L[5]));
    acc.emit(boolc(L[6]));
    acc.emit(boolc(is_real));
    const T base = k(256);
    const T overflow = sub(add(L[3], L[4]), L[1]);
    acc.emit(mul(is_real, mul(overflow, sub(overflow, base))));
    acc.emit(mul(is_real, mul(L[2], sub(overflow, base))));
    acc.emit(mul(is_real, mul(sub(L[2], one()), overflow)));
    acc.emit(mul(is_real, boolc(L[2])));
    acc.emit(mul(is_real, boolc(is_real)));
  }

  // JumpChip::eval (jump/air.rs:22-82) + IsZeroOperation::eval (operations/is_zero.rs:48-66)
  KB_HD void eval_jump() {
    const T is_real = add(L[43], L[44]);
    acc.emit(boolc(L[43]));
    acc.emit(boolc(L[44]));
    acc.emit(boolc(is_real));
    const T is_zero = sub(one(), mul(L[41], L[40]));
    acc.emit(mul(is_real, sub(is_zero, L[42])));
    acc.emit(mul(is_real, boolc(L[42])));
    acc.emit(mul(mul(is_real, L[42]), L[40]));
    const T npc = word(&L[18]), dst = word(&L[36]), pc1 = add(word(&L[0]), one());
    acc.emit(mul(mul(L[43], L[42]), sub(npc, dst)));
    acc.emit(mul(mul(L[43], sub(L[42], one())), sub(npc, pc1)));
    acc.emit(mul(mul(L[44], sub(L[42], one())), sub(npc, dst)));
    acc.emit(mul(mul(L[44], L[42]), sub(npc, pc1)));
    word_range_check(&L[0], &L[4], is_real);
    word_range_check(&L[18], &L[22], is_real);
  }

  // MemoryInstructionsChip::eval (memory/instructions/air.rs:25-76)
  KB_HD void eval_meminstrs() {
    const T is_real = add(L[38], L[39]);
    acc.emit(boolc(L[38]));
    acc.emit(boolc(L[39]));
    acc.emit(boolc(is_real));
    const T mp = word(&L[2]), nmp = word(&L[20]);
    acc.emit(mul(L[38], sub(nmp, add(mp, one()))));
    acc.emit(mul(L[39], sub(nmp, sub(mp, one()))));
    acc.emit(mul(mul(trans, N[40]), sub(nmp, word(&N[2]))));
    word_range_check(&L[2], &L[6], L[40]);
    word_range_check(&L[20], &L[24], L[40]);
  }

  // IoChip::eval (io/mod.rs:127-141)
  KB_HD void eval_io() {
    acc.emit(boolc(L[3]));
    acc.emit(boolc(L[4]));
    acc.emit(boolc(add(L[3], L[4])));
  }

  template <int CHIP>
  KB_HD void eval_air() {
    if constexpr (CHIP == 0) eval_cpu();
    else if constexpr (CHIP == 2) eval_addsub();
    else if constexpr (CHIP == 3) eval_jump();
    else if constexpr (CHIP == 6) eval_meminstrs();
    else if constexpr (CHIP == 7) eval_io();
    // Program (1), Memory (4), Byte (5): lookups only
  }

  // eval_permutation_constraints (crates/stark/src/permutation.rs:157-272).
  // perm_l / perm_n: EF columns; pa, pb: LogUp challenges; pb_pows[j] = pb^j (j <= 7).
  template <int CHIP, int J>
  KB_HD void rlc_mult(const EF& pa, const EF* pb_pows, EF& rlc, EF& mult) const {
    constexpr Lookup lk = LookupsOf<CHIP>::v.l[J];
    if constexpr (std::is_same<Ops, BaseOps>::value) {  // lazy 64-bit products (kb::LazyEF)
      kb::LazyEF lz;
      lz.init();
#pragma unroll
      for (int v = 0; v < lk.nvals; v++) lz.add(pb_pows[v + 1], vcol_eval<Ops>(lk.vals[v], PL, L));
      rlc = kb::ef_add(lz.get(), kb::ef_add(pa, kb::ef_base(kb::to_mont_c(lk.kind))));
    } else {
      EF r = kb::ef_add(pa, kb::ef_base(kb::to_mont_c(lk.kind)));
#pragma unroll
      for (int v = 0; v < lk.nvals; v++)
        r = kb::ef_add(r, Ops::mulE(pb_pows[v + 1], vcol_eval<Ops>(lk.vals[v], PL, L)));
      rlc = r;
    }
    const EF mm = Ops::toE(vcol_eval<Ops>(lk.mult, PL, L));
    mult = lk.send ? mm : kb::ef_neg(mm);
  }

  template <int CHIP, int B>
  KB_HD void perm_batch(const EF* perm_l, const EF& pa, const EF* pb_pows) {
    constexpr int NI = LookupsOf<CHIP>::v.n;
    EF r0, m0;
    rlc_mult<CHIP, 2 * B>(pa, pb_pows, r0, m0);
    EF product, numerator;
    if constexpr (2 * B + 1 < NI) {
      EF r1, m1;
      rlc_mult<CHIP, 2 * B + 1>(pa, pb_pows, r1, m1);
      product = kb::ef_mul(r0, r1);
      numerator = kb::ef_add(kb::ef_mul(m0, r1), kb::ef_mul(m1, r0));
    } else {
      product = r0;
      numerator = m0;
    }
    acc.emit_ext(kb::ef_sub(kb::ef_mul(product, perm_l[B]), numerator));
  }

  template <int CHIP, int B, int NB>
  KB_HD void perm_batches(const EF* perm_l, const EF& pa, const EF* pb_pows) {
    if constexpr (B < NB) {
      perm_batch<CHIP, B>(perm_l, pa, pb_pows);
      perm_batches<CHIP, B + 1, NB>(perm_l, pa, pb_pows);
    }
  }

  template <int CHIP>
  KB_HD void eval_perm(const EF* perm_l, const EF* perm_n, const EF& pa, const EF* pb_pows,
                       const EF& cumsum, const EF& firstE, const EF& lastE, const EF& transE) {
    constexpr int NB = (LookupsOf<CHIP>::v.n + 1) / 2;
    perm_batches<CHIP, 0, NB>(perm_l, pa, pb_pows);
    EF sum_l = kb::ef_zero(), sum_n = kb::ef_zero();
#pragma unroll
    for (int b = 0; b < NB; b++) {
      sum_l = kb::ef_add(sum_l, perm_l[b]);
      sum_n = kb::ef_add(sum_n, perm_n[b]);
    }
    const EF phi_l = perm_l[NB], phi_n = perm_n[NB];
    acc.emit_ext(kb::ef_mul(firstE, kb::ef_sub(phi_l, sum_l)));
    acc.emit_ext(kb::ef_mul(transE, kb::ef_sub(kb::ef_sub(phi_n, phi_l), sum_n)));
    acc.emit_ext(kb::ef_mul(lastE, kb::ef_sub(phi_l, cumsum)));
  }
};

// Number of constraints emitted by each chip's eval (AIR + LogUp), used to size the alpha
// power tables of the quotient kernel.
struct CountAcc {
  int n = 0;
  template <class X> KB_HD void emit(const X&) { n++; }
  KB_HD void emit_ext(const EF&) { n++; }
};

}  // namespace bfz
