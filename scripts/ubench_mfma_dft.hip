// Prototype + throughput check of a 1024-point KoalaBear DFT on the matrix cores (gfx950
// v_mfma_i32_32x32x32_i8), one wave per 1024-element block, no LDS:
//   block position p = 32 a + b holds y[bitrev10(p)]; out[k] = sum_j y[j] w^(j k), k natural.
//   j = jl + 32 jh with jl = bitrev5(a), jh = bitrev5(b); k = kl + 32 kh:
//   pass A (data = A operand, rows a, K = (b, digit)):  Z[a][kl] = sum_b M[kl][b] y(a,b)
//   twiddle Z[a][kl] *= w^(bitrev5(a) kl)
//   pass B (data = B operand straight from pass A's accumulators, K = (a, digit)):
//     out[kl + 32 kh] = sum_a M[kh][a] Z[a][kl]
//   with M[i][j] = w32^(bitrev5(j) i).  A 31-bit product is 16 int8 products: the data word is
//   split into 4 signed digits (K = 4 x 32 = 128 per element row) and the constant matrix
//   W'[i][(j, d)] = M[i][j] 2^(8d) R mod p into 4 signed digit planes (4 accumulators); the
//   planes recombine as sum_e 2^(8e) acc_e and one Montgomery reduction finishes the product.
// Build: hipcc --offload-arch=gfx950 -O3 -I zkvm-brainfuck_amd/csrc scripts/ubench_mfma_dft.hip -o /tmp/ubench_mfma_dft
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kb.h"

using namespace kb;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

// signed int8 digits of x in [-0x80808080, 0x7f7f7f7f], packed little-endian
KB_HD uint32_t digits(uint32_t x) { return (x + 0x80808080u) ^ 0x80808080u; }

// sum_e 2^(8e) acc_e (|acc_e| < 2^21) -> Montgomery reduction, result in (-p, p) as int32
__device__ __forceinline__ int32_t combine(int32_t a0, int32_t a1, int32_t a2, int32_t a3) {
  const int32_t lo = a0 + a1 * 256, hi = a2 + a3 * 256;
  const int64_t y = (int64_t)hi * 65536 + (int64_t)lo;
  const int32_t m = (int32_t)((uint32_t)y * MU_NEG);
  return (int32_t)(((int64_t)m * (int64_t)P + y) >> 32);
}

// wtab: per lane 16 v4i (plane e, K-step s at [4e + s]); ttab: per lane 16 twiddles.
template <bool LDS_W>
__global__ __launch_bounds__(256) void k_dft1024(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                 size_t nblocks, const v4i* __restrict__ wtab,
                                                 const uint32_t* __restrict__ ttab) {
  __shared__ v4i wl[LDS_W ? 64 * 16 : 1];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  v4i W[16];
  if constexpr (LDS_W) {
    for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) wl[i] = wtab[i];
    __syncthreads();
  } else {
#pragma unroll
    for (int i = 0; i < 16; i++) W[i] = wtab[lane * 16 + i];
  }
  uint32_t tw[16];
#pragma unroll
  for (int q = 0; q < 16; q++) tw[q] = ttab[lane * 16 + q];
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t blk = wave; blk < nblocks; blk += nw) {
    const uint32_t* X = in + blk * 1024;
    v4i A[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint4 v = *reinterpret_cast<const uint4*>(X + 32 * r + 8 * s + 4 * h);
      A[s] = v4i{(int)digits(v.x), (int)digits(v.y), (int)digits(v.z), (int)digits(v.w)};
    }
    v16i acc[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      acc[e] = v16i{};
#pragma unroll
      for (int s = 0; s < 4; s++) {
        const v4i w = LDS_W ? wl[lane * 16 + 4 * e + s] : W[4 * e + s];
        acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], w, acc[e], 0, 0, 0);
      }
    }
    v4i B[4];
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int32_t z = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
      const uint32_t zt = mmul_s(z, tw[q]);  // [0, p)
      B[q >> 2][q & 3] = (int)digits(zt);
    }
#pragma unroll
    for (int e = 0; e < 4; e++) {
      acc[e] = v16i{};
#pragma unroll
      for (int s = 0; s < 4; s++) {
        const v4i w = LDS_W ? wl[lane * 16 + 4 * e + s] : W[4 * e + s];
        acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w, B[s], acc[e], 0, 0, 0);
      }
    }
    uint32_t* Y = out + blk * 1024;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int32_t y = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
      const uint32_t yc = umin((uint32_t)y, (uint32_t)y + P);
      const int kh = (q & 3) + 8 * (q >> 2) + 4 * h;
      Y[r + 32 * kh] = yc;
    }
  }
}

// Natural in -> bit-reversed out (the DIF tile's inner 1024 points):
//   n = nl + 32 nh, k = k1 + 32 k2; pass A rows nl, K = (nh, digit): Z[nl][k1] = sum_nh M[k1][nh] z
//   twiddle w^(nl k1); pass B: out[bitrev5(k1) 32 + rho] = sum_nl M2[rho][nl] Z'[nl][k1] with
//   M2[rho][nl] = w32^(nl bitrev5(rho)) (rows in bit-reversed order) and M[k1][nh] = w32^(nh k1).
// wtab2: [0, 16) pass-A planes (M), [16, 32) pass-B planes (M2).
__global__ __launch_bounds__(256) void k_dft1024_dif(const uint32_t* __restrict__ in,
                                                     uint32_t* __restrict__ out, size_t nblocks,
                                                     const v4i* __restrict__ wtab2,
                                                     const uint32_t* __restrict__ ttab) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  uint32_t tw[16];
#pragma unroll
  for (int q = 0; q < 16; q++) tw[q] = ttab[lane * 16 + q];
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const v4i* WL = wtab2 + lane * 32;
  for (size_t blk = wave; blk < nblocks; blk += nw) {
    const uint32_t* X = in + blk * 1024;
    v4i A[4];
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int t = 0; t < 4; t++) A[s][t] = (int)digits(X[r + 32 * (8 * s + 4 * h + t)]);
    v16i acc[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      acc[e] = v16i{};
#pragma unroll
      for (int s = 0; s < 4; s++) acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], WL[4 * e + s], acc[e], 0, 0, 0);
    }
    v4i B[4];
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int32_t z = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
      B[q >> 2][q & 3] = (int)digits(mmul_s(z, tw[q]));
    }
#pragma unroll
    for (int e = 0; e < 4; e++) {
      acc[e] = v16i{};
#pragma unroll
      for (int s = 0; s < 4; s++) acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(WL[16 + 4 * e + s], B[s], acc[e], 0, 0, 0);
    }
    uint32_t* Y = out + blk * 1024 + 32 * (__builtin_bitreverse32((uint32_t)r) >> 27);
#pragma unroll
    for (int g = 0; g < 4; g++) {
      uint4 v;
      uint32_t o[4];
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int32_t y = combine(acc[0][4 * g + t], acc[1][4 * g + t], acc[2][4 * g + t], acc[3][4 * g + t]);
        o[t] = umin((uint32_t)y, (uint32_t)y + P);
      }
      v = uint4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<uint4*>(Y + 8 * g + 4 * h) = v;
    }
  }
}

// V2: constants streamed from LDS inside the loop (an opaque zero stops the compiler hoisting
// 80 registers of loop invariants), accumulators at most 64 registers, WPE waves per SIMD.
template <int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_dft1024_v2(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t nblocks,
    const v4i* __restrict__ wtab, const uint32_t* __restrict__ ttab) {
  __shared__ v4i wl[64 * 16];
  __shared__ uint32_t tl[64 * 16];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
    wl[(i & 15) * 64 + (i >> 4)] = wtab[i];  // [reg][lane]: a wave reads 64 consecutive entries
    tl[(i & 15) * 64 + (i >> 4)] = ttab[i];
  }
  __syncthreads();
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t blk = wave; blk < nblocks; blk += nw) {
    const int z = (int)opaque(0u);
    const v4i* WL = wl + lane + z;
    const uint32_t* TL = tl + lane + z;
    const uint32_t* X = in + blk * 1024;
    v4i A[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint4 v = *reinterpret_cast<const uint4*>(X + 32 * r + 8 * s + 4 * h);
      A[s] = v4i{(int)digits(v.x), (int)digits(v.y), (int)digits(v.z), (int)digits(v.w)};
    }
    v16i acc[4];
#pragma unroll
    for (int e = 0; e < 4; e++) acc[e] = v16i{};
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int e = 0; e < 4; e++) acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], WL[64 * (4 * e + s)], acc[e], 0, 0, 0);
    v4i B[4];
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int32_t zz = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
      B[q >> 2][q & 3] = (int)digits(mmul_s(zz, TL[64 * q]));
    }
#pragma unroll
    for (int e = 0; e < 4; e++) acc[e] = v16i{};
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int e = 0; e < 4; e++) acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(WL[64 * (4 * e + s)], B[s], acc[e], 0, 0, 0);
    uint32_t* Y = out + blk * 1024;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int32_t y = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
      const int kh = (q & 3) + 8 * (q >> 2) + 4 * h;
      Y[r + 32 * kh] = umin((uint32_t)y, (uint32_t)y + P);
    }
  }
}

// Compute-only rate: the same two passes REPS times on register data per block (the output
// digits are fed back as the next A operand: not a DFT of anything, the same instructions).
template <int REPS>
__global__ __launch_bounds__(256) void k_dft1024_reps(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      size_t nblocks, const v4i* __restrict__ wtab,
                                                      const uint32_t* __restrict__ ttab) {
  __shared__ v4i wl[64 * 16];
  __shared__ uint32_t tl[64 * 16];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
    wl[(i & 15) * 64 + (i >> 4)] = wtab[i];  // [reg][lane]: a wave reads 64 consecutive entries
    tl[(i & 15) * 64 + (i >> 4)] = ttab[i];
  }
  __syncthreads();
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t blk = wave; blk < nblocks; blk += nw) {
    const uint32_t* X = in + blk * 1024;
    v4i A[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint4 v = *reinterpret_cast<const uint4*>(X + 32 * r + 8 * s + 4 * h);
      A[s] = v4i{(int)digits(v.x), (int)digits(v.y), (int)digits(v.z), (int)digits(v.w)};
    }
    uint32_t o[16];
#pragma nounroll
    for (int rep = 0; rep < REPS; rep++) {
      const int z = (int)opaque(0u);
      const v4i* WL = wl + lane + z;
      const uint32_t* TL = tl + lane + z;
      v16i acc[4];
#pragma unroll
      for (int e = 0; e < 4; e++) acc[e] = v16i{};
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int e = 0; e < 4; e++) acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], WL[64 * (4 * e + s)], acc[e], 0, 0, 0);
      v4i B[4];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int32_t zz = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
        B[q >> 2][q & 3] = (int)digits(mmul_s(zz, TL[64 * q]));
      }
#pragma unroll
      for (int e = 0; e < 4; e++) acc[e] = v16i{};
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int e = 0; e < 4; e++) acc[e] = __builtin_amdgcn_mfma_i32_32x32x32_i8(WL[64 * (4 * e + s)], B[s], acc[e], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int32_t y = combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
        o[q] = umin((uint32_t)y, (uint32_t)y + P);
        A[q >> 2][q & 3] = (int)digits(o[q]);
      }
    }
    uint32_t* Y = out + blk * 1024;
#pragma unroll
    for (int q = 0; q < 16; q++) Y[r + 32 * ((q & 3) + 8 * (q >> 2) + 4 * h)] = o[q];
  }
}

// VALU reference: 16 elements per thread, REPS x (two radix-16 windows of 4 DIT stages + a
// twiddle) ~ the existing r16 arithmetic, 8 stages per rep on registers.
template <int REPS>
__global__ __launch_bounds__(256) void k_valu_reps(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                   size_t n) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t T = (size_t)gridDim.x * blockDim.x;
  for (size_t base = t; base * 16 < n; base += T) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = in[base * 16 + i];
    uint32_t tw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) tw[i] = (uint32_t)((base + i) * 40503u) % P;
#pragma nounroll
    for (int rep = 0; rep < REPS; rep++) {
#pragma unroll
      for (int kk = 0; kk < 4; kk++)
#pragma unroll
        for (int i = 0; i < 16; i++) {
          if (i & (1 << kk)) continue;
          const int j = i | (1 << kk);
          const uint32_t vw = mmul(x[j], tw[i & 7]);
          const uint32_t s_ = x[i] + vw, d = x[i] - vw;
          x[i] = umin(s_, s_ - P);
          x[j] = umin(d, d + P);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; i++) out[base * 16 + i] = x[i];
  }
}

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

static int bitrev(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

int main(int argc, char** argv) {
  const int logblocks = argc > 1 ? std::atoi(argv[1]) : 16;  // 2^16 blocks = 2^26 elements
  const size_t nblocks = (size_t)1 << logblocks, n = nblocks * 1024;
  const uint32_t w = two_adic_gen(10);  // Montgomery
  const uint32_t w32 = mpow(w, 32);
  // M[i][j] = w32^(bitrev5(j) i), Montgomery; W'[i][(j,d)] = M[i][j] 2^(8d) R (Montgomery of
  // M 2^(8d), times R once more so that the reduction of the recombined planes is exact)
  std::vector<v4i> wtab(64 * 16);
  std::vector<uint32_t> ttab(64 * 16);
  for (int lane = 0; lane < 64; lane++) {
    const int rr = lane & 31, h = lane >> 5;
    for (int e = 0; e < 4; e++)
      for (int s = 0; s < 4; s++) {
        int8_t bytes[16];
        for (int j = 0; j < 16; j++) {
          const int jj = 8 * s + 4 * h + (j >> 2), d = j & 3;
          const uint32_t m = mpow(w32, (uint64_t)bitrev(jj, 5) * rr);  // Montgomery word M R
          // V = M 2^(8d) R mod p (the residue; mmul by R2 multiplies by R, from_mont divides)
          const uint32_t V = from_mont(mmul(mmul(m, to_mont(1u << (8 * d))), R2));
          const uint32_t dg = digits(V);
          bytes[j] = (int8_t)(dg >> (8 * e));
        }
        v4i x;
        std::memcpy(&x, bytes, 16);
        wtab[lane * 16 + 4 * e + s] = x;
      }
    for (int q = 0; q < 16; q++) {
      const int a = (q & 3) + 8 * (q >> 2) + 4 * h;
      ttab[lane * 16 + q] = mpow(w, (uint64_t)bitrev(a, 5) * rr);
    }
  }
  // DIF tables: [0, 16) pass A (M[k1][nh] = w32^(nh k1)), [16, 32) pass B (M2[rho][nl] =
  // w32^(nl bitrev5(rho))); twiddles w^(nl k1)
  std::vector<v4i> wtab2(64 * 32);
  std::vector<uint32_t> ttab2(64 * 16);
  for (int lane = 0; lane < 64; lane++) {
    const int rr = lane & 31, h = lane >> 5;
    for (int pass = 0; pass < 2; pass++)
      for (int e = 0; e < 4; e++)
        for (int s = 0; s < 4; s++) {
          int8_t bytes[16];
          for (int j = 0; j < 16; j++) {
            const int jj = 8 * s + 4 * h + (j >> 2), d = j & 3;
            const uint64_t ex = pass == 0 ? (uint64_t)jj * rr : (uint64_t)jj * bitrev(rr, 5);
            const uint32_t m = mpow(w32, ex);
            const uint32_t V = from_mont(mmul(mmul(m, to_mont(1u << (8 * d))), R2));
            bytes[j] = (int8_t)(digits(V) >> (8 * e));
          }
          v4i x;
          std::memcpy(&x, bytes, 16);
          wtab2[lane * 32 + 16 * pass + 4 * e + s] = x;
        }
    for (int q = 0; q < 16; q++) {
      const int nl = (q & 3) + 8 * (q >> 2) + 4 * h;
      ttab2[lane * 16 + q] = mpow(w, (uint64_t)nl * rr);
    }
  }
  std::vector<uint32_t> hin(n);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < n; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    hin[i] = (uint32_t)(s % P);
  }
  uint32_t *din, *dout;
  v4i* dw;
  uint32_t* dt;
  CK(hipMalloc(&din, n * 4));
  CK(hipMalloc(&dout, n * 4));
  CK(hipMalloc(&dw, wtab.size() * sizeof(v4i)));
  CK(hipMalloc(&dt, ttab.size() * 4));
  CK(hipMemcpy(din, hin.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, wtab.data(), wtab.size() * sizeof(v4i), hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ttab.data(), ttab.size() * 4, hipMemcpyHostToDevice));
  v4i* dw2;
  uint32_t* dt2;
  CK(hipMalloc(&dw2, wtab2.size() * sizeof(v4i)));
  CK(hipMalloc(&dt2, ttab2.size() * 4));
  CK(hipMemcpy(dw2, wtab2.data(), wtab2.size() * sizeof(v4i), hipMemcpyHostToDevice));
  CK(hipMemcpy(dt2, ttab2.data(), ttab2.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch, const char* what, double elem_stages, double bytes) {
    launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; i++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::printf("%-28s %8.1f us  %6.2f T elem-stages/s  %7.1f GB/s\n", what, ms * 1e3,
                elem_stages / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 1e9);
  };
  const double es = (double)n * 10, by = 8.0 * n;
  for (int grid : {1024, 2048, 4096, 8192}) {
    char name[64];
    std::snprintf(name, sizeof name, "mfma regW grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024<false>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, es, by);
    std::snprintf(name, sizeof name, "mfma ldsW grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024<true>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, es, by);
  }
  for (int grid : {2048, 4096, 8192}) {
    char name[64];
    std::snprintf(name, sizeof name, "mfma v2 wpe2 grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024_v2<2>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, es, by);
    std::snprintf(name, sizeof name, "mfma v2 wpe3 grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024_v2<3>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, es, by);
    std::snprintf(name, sizeof name, "mfma v2 wpe4 grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024_v2<4>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, es, by);
  }
  for (int grid : {2048, 4096}) {
    char name[64];
    std::snprintf(name, sizeof name, "mfma reps1 grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024_reps<1>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, es, by);
    std::snprintf(name, sizeof name, "mfma reps5 grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024_reps<5>, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw, dt); },
         name, 5 * es, by);
    std::snprintf(name, sizeof name, "valu reps1 (4 st) grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_valu_reps<1>, dim3(grid), dim3(256), 0, 0, din, dout, n); },
         name, (double)n * 4, by);
    std::snprintf(name, sizeof name, "valu reps5 (4 st) grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_valu_reps<5>, dim3(grid), dim3(256), 0, 0, din, dout, n); },
         name, (double)n * 20, by);
  }
  for (int grid : {2048, 4096}) {
    char name[64];
    std::snprintf(name, sizeof name, "mfma dif grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_dft1024_dif, dim3(grid), dim3(256), 0, 0, din, dout, nblocks, dw2, dt2); },
         name, es, by);
  }
  time([&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (const uint4*)din, (uint4*)dout, n / 4); },
       "copy", 0, by);
  // correctness: a few blocks against the O(n^2) DFT
  hipLaunchKernelGGL(k_dft1024<false>, dim3(2048), dim3(256), 0, 0, din, dout, nblocks, dw, dt);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hout(n);
  CK(hipMemcpy(hout.data(), dout, n * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (size_t blk : {(size_t)0, (size_t)1, nblocks / 3, nblocks - 1}) {
    const uint32_t* X = &hin[blk * 1024];
    for (int k = 0; k < 1024; k++) {
      uint32_t acc = 0, wk = mpow(w, (uint64_t)k), p = ONE;
      for (int j = 0; j < 1024; j++) {
        acc = madd(acc, mmul(X[bitrev(j, 10)], p));
        p = mmul(p, wk);
      }
      bad += acc != hout[blk * 1024 + k];
    }
  }
  std::printf("check (bitrev in, natural out): %d of 4096 outputs wrong\n", bad);
  {
    std::vector<uint32_t> ref = hout;
    hipLaunchKernelGGL(k_dft1024_v2<4>, dim3(2048), dim3(256), 0, 0, din, dout, nblocks, dw, dt);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hout.data(), dout, n * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < n; i++) diff += hout[i] != ref[i];
    std::printf("check v2 == v1 over all %zu outputs: %zu differ\n", n, diff);
    bad += diff != 0;
  }
  hipLaunchKernelGGL(k_dft1024_dif, dim3(2048), dim3(256), 0, 0, din, dout, nblocks, dw2, dt2);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hout.data(), dout, n * 4, hipMemcpyDeviceToHost));
  int bad2 = 0;
  for (size_t blk : {(size_t)0, (size_t)1, nblocks / 3, nblocks - 1}) {
    const uint32_t* X = &hin[blk * 1024];
    for (int k = 0; k < 1024; k++) {
      uint32_t acc = 0, wk = mpow(w, (uint64_t)k), p = ONE;
      for (int j = 0; j < 1024; j++) {
        acc = madd(acc, mmul(X[j], p));
        p = mmul(p, wk);
      }
      bad2 += acc != hout[blk * 1024 + bitrev(k, 10)];
    }
  }
  std::printf("check (natural in, bitrev out): %d of 4096 outputs wrong\n", bad2);
  return bad + bad2 != 0;
}
