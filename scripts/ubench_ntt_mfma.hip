// Matrix-core 2^14-point NTT tiles: measured and dropped, kept as a standalone
// microbenchmark.  Round 4 shipped them in libbfz behind BFZ_NTT_MFMA=1; they are bit-exact but
// slower than the VALU tiles (DIT 205 vs 176 us, DIF 232 vs 189 us per 2^26-element pass), so the
// product library no longer carries them.  This program runs both on the same 2^26 words and
// checks that the outputs are identical (the VALU tile is bfz::ntt_passes with L = 14).
// Build (links the product library for ntt_passes, the twiddle tables and the stream):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zkvm-brainfuck_amd/csrc scripts/ubench_ntt_mfma.hip \
//     -L zkvm-brainfuck_amd -lbfz -Wl,-rpath,'$ORIGIN/../zkvm-brainfuck_amd' -o scripts/ubench_ntt_mfma
// Diagnostic builds: -DBFZ_MF_DIAG=1 (no 1024-point transforms: data movement + the radix-16
// window) or 2 (no radix-16 window); their outputs are wrong by construction.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "gpu.h"
#include "ntt.h"
#include "ntt_dev.h"

namespace bfz {

// ---------------------------------------------------------------------------------------
// 2^14-point tile passes with ten of the fourteen stages on the matrix cores (gfx950
// v_mfma_i32_32x32x32_i8).  A 1024-point DFT with a root w of order 1024 is two 32-point
// DFTs and a twiddle (j = jl + 32 jh, k = kl + 32 kh:  w^(jk) = w^(jl kl) w32^(jl kh) w32^(jh kl)),
// and a 32-point DFT of 32 rows is a 32 x 32 matrix product.  A 31-bit product is 16 int8
// products: each data word is split into 4 signed digits (x = sum_d x_d 2^(8d), K = 32 words
// x 4 digits = 4 MFMA K-steps) and the constant matrix entry into the 4 signed digit planes of
// V_d = M 2^(8d) R mod p (4 accumulators e); sum_e 2^(8e) acc_e = sum_j M_j x_j R (mod p) as an
// exact 64-bit integer (|acc_e| < 2^21), and one signed Montgomery reduction gives the
// Montgomery product.  Per element that is ~36 VALU units for ten stages against ~75 for ten
// radix-2 stages (the 32 MFMAs per 1024 elements run on the matrix pipe beside them).
//   DIT tile (bit-reversed in, natural out):  wave b transforms block b (positions
//     [1024 b, 1024 b + 1024) hold the bit-reversed 1024-point subsequence: stages 0..9 are its
//     DFT), results to LDS; then the radix-16 window g0 = 10 (stages 10..13) as k_ntt_tile's
//     and straight to HBM.
//   DIF tile (natural in, bit-reversed out): the radix-16 window g0 = 10 (stages 13..10) on
//     elements tid + 1024 i straight from HBM, to LDS; then wave b runs stages 9..0 = the
//     1024-point DFT of block b, natural in, bit-reversed out, straight to HBM.
// The MFMA layouts (v_mfma_i32_32x32x32_i8, wave64): A operand lane l = row l & 31, K bytes
// [16 (l >> 5), +16); B operand lane l = column l & 31, same K split; accumulator element q of
// lane l = row (q & 3) + 8 (q >> 2) + 4 (l >> 5), column l & 31.  Pass A's accumulator is
// therefore pass B's B operand with no lane exchange (scripts/ubench_mfma_dft.hip checks both
// directions against an O(n^2) DFT).
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t i8_digits(uint32_t x) {  // x < 0x7f7f7f7f
  return (x + 0x80808080u) ^ 0x80808080u;
}
// sum_e 2^(8e) acc_e, Montgomery-reduced: result in (-p, p) as int32
__device__ __forceinline__ int32_t mfma_combine(int32_t a0, int32_t a1, int32_t a2, int32_t a3) {
  const int32_t lo = a0 + a1 * 256, hi = a2 + a3 * 256;
  const int64_t y = (int64_t)hi * 65536 + (int64_t)lo;
  const int32_t m = (int32_t)((uint32_t)y * MU_NEG);
  return (int32_t)(((int64_t)m * (int64_t)P + y) >> 32);
}

constexpr int MF_DATA = 1 << 14;  // LDS words of tile data (64 KiB: two tiles per CU)
constexpr int MF_THREADS = 512;   // 8 waves, two 1024-point blocks each
// DIT: the 16 KiB table staged in LDS per block (64 + 16 KiB: still two tiles per CU; -24% against
// reading it through L1/L2); the DIF's two tables (32 KiB) are read from L1/L2.
constexpr bool MF_LDSW = true;
#ifndef BFZ_MF_DIAG
#define BFZ_MF_DIAG 0  // diagnostic builds: 1 = no 1024-point transforms, 2 = no radix-16 window
#endif

// The constant tables live in global memory (L1/L2-resident, 16 or 32 KiB) in [reg][lane]
// order: one register of the table is 64 consecutive v4i, one coalesced 1 KiB wave load.
typedef const __attribute__((address_space(1))) v4i gv4i;
typedef const __attribute__((address_space(1))) uint32_t gu32;
// a zero the compiler cannot see through or merge with another (volatile: never CSE'd), so
// each use of a table is a fresh load instead of registers held across the kernel
__device__ __forceinline__ uint32_t fresh_zero() {
  uint32_t z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

// 16 MFMAs: acc_e = sum_s X[s] x W[e][s] (data as the A operand) or W[e][s] x X[s] (as B);
// out[q] = Montgomery(sum_e 2^(8e) acc_e) in (-p, p).  The table registers of each K-step are
// read afresh (4 in flight, not the whole 16-register table held across the kernel).
// (Two accumulator groups of two planes each, 32 registers instead of 64, measured slower.)
template <bool DATA_IS_A, class TW>
__device__ __forceinline__ void mf_pass(int32_t (&out)[16], const v4i (&X)[4], TW* __restrict__ W) {
  v16i acc[4];
#pragma unroll
  for (int e = 0; e < 4; e++) acc[e] = v16i{};
#pragma unroll
  for (int s = 0; s < 4; s++) {
    TW* WL = W + fresh_zero();
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const v4i w = WL[64 * (4 * e + s)];
      acc[e] = DATA_IS_A ? __builtin_amdgcn_mfma_i32_32x32x32_i8(X[s], w, acc[e], 0, 0, 0)
                         : __builtin_amdgcn_mfma_i32_32x32x32_i8(w, X[s], acc[e], 0, 0, 0);
    }
  }
#pragma unroll
  for (int q = 0; q < 16; q++) out[q] = mfma_combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
}
// pass A -> twiddle -> pass B on one 1024-point block; X: the block's digits (A operand);
// out: the transform in (-p, p), element q of lane l at pass B's accumulator position
template <class TW>
__device__ __forceinline__ void mf_dft1024(int32_t (&out)[16], v4i (&X)[4], TW* __restrict__ WA,
                                           TW* __restrict__ WB, gu32* __restrict__ TL) {
#if BFZ_MF_DIAG == 1  // diagnostic: no transform (data movement + the radix-16 window)
#pragma unroll
  for (int q = 0; q < 16; q++) out[q] = X[q >> 2][q & 3] & 0x3fffffff;
  return;
#endif
  mf_pass<true>(out, X, WA);
#pragma unroll
  for (int q = 0; q < 16; q++) X[q >> 2][q & 3] = (int)i8_digits(mmul_s(out[q], TL[64 * q]));
  mf_pass<false>(out, X, WB);
}

template <bool DIF>
__global__ __launch_bounds__(MF_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_tile14_mfma(
    const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, size_t src_stride, size_t dst_stride,
    const uint32_t* __restrict__ tw, const v4i* __restrict__ wtab, const uint32_t* __restrict__ ttab) {
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const size_t base = (size_t)blockIdx.x << 14;
  const uint32_t* S = src + (size_t)blockIdx.y * src_stride + base;
  uint32_t* D = dst + (size_t)blockIdx.y * dst_stride + base;
  gv4i* WA = (gv4i*)wtab + lane;
  gv4i* WB = WA + (DIF ? 64 * 16 : 0);
  gu32* TL = (gu32*)ttab + lane;
  v4i* wl = reinterpret_cast<v4i*>(lds + MF_DATA);
  if constexpr (!DIF && MF_LDSW) {
    for (int i = tid; i < 16 * 64; i += MF_THREADS) wl[i] = ((gv4i*)wtab)[i];
    __syncthreads();
  }
  int32_t y[16];
  if constexpr (!DIF) {
#pragma nounroll
    for (int k = 0; k < 2; k++) {  // (unrolled: neutral)
      const uint32_t* Xg = S + (wave + 8 * k) * 1024;
      v4i X[4];
#pragma unroll
      for (int s = 0; s < 4; s++) {
        const uint4 v = *reinterpret_cast<const uint4*>(Xg + 32 * r + 8 * s + 4 * h);
        X[s] = v4i{(int)i8_digits(v.x), (int)i8_digits(v.y), (int)i8_digits(v.z), (int)i8_digits(v.w)};
      }
      if constexpr (MF_LDSW)
        mf_dft1024(y, X, (const v4i*)wl + lane, (const v4i*)wl + lane, TL);
      else
        mf_dft1024(y, X, WA, WB, TL);
      uint32_t* blk = lds + (wave + 8 * k) * 1024;
#pragma unroll
      for (int q = 0; q < 16; q++)
        blk[r + 32 * ((q & 3) + 8 * (q >> 2) + 4 * h)] = umin((uint32_t)y[q], (uint32_t)y[q] + P);
    }
    __syncthreads();
#pragma nounroll
    for (int k = 0; k < 2; k++) {
      const int c = tid + MF_THREADS * k;
      uint32_t x[16];
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = lds[c + 1024 * i];
#if BFZ_MF_DIAG != 2
      r16_window<false, false, true, 4>(x, 10, 0, 4, 0, (uint32_t)c, 0, tw);
#endif
#pragma unroll
      for (int i = 0; i < 16; i++) D[c + 1024 * i] = x[i];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int c = tid + MF_THREADS * k;
      uint32_t x[16];
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = S[c + 1024 * i];
#if BFZ_MF_DIAG != 2
      r16_window<true, false, true, 4>(x, 10, 0, 4, 0, (uint32_t)c, 0, tw);
#endif
#pragma unroll
      for (int i = 0; i < 16; i++) lds[c + 1024 * i] = x[i];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t* blk = lds + (wave + 8 * k) * 1024;
      v4i X[4];
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int t = 0; t < 4; t++) X[s][t] = (int)i8_digits(blk[r + 32 * (8 * s + 4 * h + t)]);
      mf_dft1024(y, X, WA, WB, TL);
      uint32_t* Y = D + (wave + 8 * k) * 1024 + 32 * (__builtin_bitreverse32((uint32_t)r) >> 27);
#pragma unroll
      for (int g = 0; g < 4; g++) {
        uint32_t o[4];
#pragma unroll
        for (int t = 0; t < 4; t++) o[t] = umin((uint32_t)y[4 * g + t], (uint32_t)y[4 * g + t] + P);
        *reinterpret_cast<uint4*>(Y + 8 * g + 4 * h) = uint4{o[0], o[1], o[2], o[3]};
      }
    }
  }
}

// Host tables of the 1024-point DFTs (root w of order 1024, Montgomery):
//   DIT: [pass A = pass B] M[i][j] = w32^(bitrev5(j) i);  twiddle lane (i, h), q: w^(bitrev5(a) i)
//   DIF: pass A F[i][j] = w32^(j i), pass B M2[i][j] = w32^(j bitrev5(i));  twiddle w^(a i)
// with a = (q & 3) + 8 (q >> 2) + 4 h.  Table entry [16 pass + 4 e + s][lane] holds, for K byte
// kb (j = 8 s + 4 h + kb / 4, d = kb % 4), digit e of V = M[lane & 31][j] 2^(8d) R mod p.
struct MfmaTables {
  DBuf<v4i> w_dit, w_dif;
  DBuf<uint32_t> t_dit, t_dif;
  bool ready = false;
};
static int brev(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}
static MfmaTables& mfma_tables() {
  static MfmaTables T;
  if (T.ready) return T;
  for (int dif = 0; dif < 2; dif++) {
    const uint32_t w = dif ? two_adic_gen(10) : minv(two_adic_gen(10));
    const uint32_t w32 = mpow(w, 32);
    const int NT = dif ? 2 : 1;
    std::vector<v4i> wt(64 * 16 * NT);
    std::vector<uint32_t> tt(64 * 16);
    for (int lane = 0; lane < 64; lane++) {
      const int i = lane & 31, h = lane >> 5;
      for (int pass = 0; pass < NT; pass++)
        for (int e = 0; e < 4; e++)
          for (int s = 0; s < 4; s++) {
            int8_t bytes[16];
            for (int kb = 0; kb < 16; kb++) {
              const int j = 8 * s + 4 * h + kb / 4, d = kb % 4;
              const uint64_t ex = !dif ? (uint64_t)brev(j, 5) * i
                                       : (pass == 0 ? (uint64_t)j * i : (uint64_t)j * brev(i, 5));
              const uint32_t m = mpow(w32, ex);
              const uint32_t V = from_mont(mmul(mmul(m, to_mont(1u << (8 * d))), R2));
              bytes[kb] = (int8_t)(((V + 0x80808080u) ^ 0x80808080u) >> (8 * e));
            }
            std::memcpy(&wt[(16 * pass + 4 * e + s) * 64 + lane], bytes, 16);
          }
      for (int q = 0; q < 16; q++) {
        const int a = (q & 3) + 8 * (q >> 2) + 4 * h;
        tt[q * 64 + lane] = mpow(w, (uint64_t)(dif ? a : brev(a, 5)) * i);
      }
    }
    DBuf<v4i>& dw = dif ? T.w_dif : T.w_dit;
    DBuf<uint32_t>& dt = dif ? T.t_dif : T.t_dit;
    dw.reset(wt.size());
    dt.reset(tt.size());
    HIP_CHECK(hipMemcpyAsync(dw.p, wt.data(), wt.size() * sizeof(v4i), hipMemcpyHostToDevice, stream()));
    HIP_CHECK(hipMemcpyAsync(dt.p, tt.data(), tt.size() * 4, hipMemcpyHostToDevice, stream()));
  }
  HIP_CHECK(hipStreamSynchronize(stream()));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tile14_mfma<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, MF_DATA * 4 + (MF_LDSW ? 16384 : 0)));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tile14_mfma<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, MF_DATA * 4));
  T.ready = true;
  return T;
}

}  // namespace bfz

using namespace bfz;

int main() {
  const int L = 14, W = 4096;  // 4096 columns of 2^14: 2^26 words
  const size_t n = (size_t)1 << L, words = n * W;
  hipStream_t st = stream();
  twiddles().ensure(L);
  uint32_t *a, *ref, *out;
  HIP_CHECK(hipMalloc(&a, words * 4));
  HIP_CHECK(hipMalloc(&ref, words * 4));
  HIP_CHECK(hipMalloc(&out, words * 4));
  std::vector<uint32_t> h(words);
  for (size_t i = 0; i < words; i++) h[i] = (uint32_t)((i * 2654435761u) % P);
  HIP_CHECK(hipMemcpy(a, h.data(), words * 4, hipMemcpyHostToDevice));
  MfmaTables& M = mfma_tables();
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  int bad = 0;
  for (int dif = 0; dif < 2; dif++) {
    const uint32_t* tw = dif ? twiddles().fwd() : twiddles().inv();
    auto mfma = [&] {
      if (dif)
        hipLaunchKernelGGL(k_tile14_mfma<true>, dim3(1, W), dim3(MF_THREADS), MF_DATA * 4, st, a, out,
                           n, n, tw, (const v4i*)M.w_dif.p, (const uint32_t*)M.t_dif.p);
      else
        hipLaunchKernelGGL(k_tile14_mfma<false>, dim3(1, W), dim3(MF_THREADS),
                           MF_DATA * 4 + (MF_LDSW ? 16384 : 0), st, a, out, n, n, tw,
                           (const v4i*)M.w_dit.p, (const uint32_t*)M.t_dit.p);
    };
    auto valu = [&] { ntt_passes(a, ref, n, n, W, L, dif, st); };
    double us[2];
    for (int k = 0; k < 2; k++) {
      auto run = [&] { k ? mfma() : valu(); };
      run();
      HIP_CHECK(hipStreamSynchronize(st));
      const int reps = 20;
      HIP_CHECK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; r++) run();
      HIP_CHECK(hipEventRecord(e1, st));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      us[k] = ms * 1e3 / reps;
    }
    std::vector<uint32_t> r1(words), r2(words);
    HIP_CHECK(hipMemcpy(r1.data(), ref, words * 4, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(r2.data(), out, words * 4, hipMemcpyDeviceToHost));
    const bool same = std::memcmp(r1.data(), r2.data(), words * 4) == 0;
    bad += !same;
    std::printf("%s 2^14 tiles x %d: VALU %.1f us, MFMA %.1f us, outputs %s\n", dif ? "DIF" : "DIT",
                W, us[0], us[1], same ? "identical" : "DIFFER");
  }
  return BFZ_MF_DIAG == 0 ? bad : 0;
}
