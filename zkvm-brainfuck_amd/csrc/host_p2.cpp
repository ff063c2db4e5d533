// Host Poseidon2KoalaBear<16> for the transcript (DuplexChallenger) and the verifier.
//
// The prover's Fiat-Shamir transcript runs on the host between device stages: after the
// openings it observes every opened value (~2,200 words = ~270 sequential permutations per
// FIBO_X4 proof) while the GPU waits for the FRI batching challenge.  The scalar permutation
// (poseidon2.h, shared with the device) takes ~1.4 us; this AVX-512 form keeps the whole
// 16-element state in one zmm register: the S-box, the diagonal and the M4 blocks run on all
// lanes at once, the block and lane sums are in-register shuffles.  Same constants and the
// same round structure as poseidon2_permute_lane (canonical Montgomery values in [0, p)); the
// result is checked against the scalar permutation once per process before it is used.
#include <immintrin.h>

#include <cstring>
#include <stdexcept>

#include "poseidon2.h"

namespace bfz {

namespace {

#define BFZ_AVX512 __attribute__((target("avx512f")))

BFZ_AVX512 inline __m512i v_p() { return _mm512_set1_epi32((int)kb::P); }

// Montgomery product of canonical values (p < 2^31): t + m p < 2^64 is a multiple of 2^32
// whose high word lies in [0, 2p); one min() makes it canonical.
BFZ_AVX512 inline __m512i v_mul(__m512i a, __m512i b) {
  const __m512i mun = _mm512_set1_epi32((int)kb::MU_NEG);
  const __m512i ao = _mm512_srli_epi64(a, 32), bo = _mm512_srli_epi64(b, 32);
  const __m512i te = _mm512_mul_epu32(a, b), to = _mm512_mul_epu32(ao, bo);
  const __m512i qe = _mm512_mul_epu32(_mm512_mul_epu32(te, mun), v_p());
  const __m512i qo = _mm512_mul_epu32(_mm512_mul_epu32(to, mun), v_p());
  const __m512i re = _mm512_add_epi64(te, qe), ro = _mm512_add_epi64(to, qo);
  const __m512i r = _mm512_mask_blend_epi32(0xAAAA, _mm512_srli_epi64(re, 32), ro);
  return _mm512_min_epu32(r, _mm512_sub_epi32(r, v_p()));
}

BFZ_AVX512 inline __m512i v_add(__m512i a, __m512i b) {
  const __m512i s = _mm512_add_epi32(a, b);  // < 2p < 2^32
  return _mm512_min_epu32(s, _mm512_sub_epi32(s, v_p()));
}

BFZ_AVX512 inline __m512i v_cube(__m512i x) { return v_mul(v_mul(x, x), x); }

// M4 = [[2,3,1,1],[1,2,3,1],[1,1,2,3],[3,1,1,2]] on each 128-bit lane (4-element block), then
// each element gets the sum of the four blocks at its position.
BFZ_AVX512 inline __m512i v_mds_light(__m512i x) {
  const __m512i x1 = _mm512_shuffle_epi32(x, (_MM_PERM_ENUM)0x39);  // x_(j+1 mod 4)
  const __m512i x2 = _mm512_shuffle_epi32(x, (_MM_PERM_ENUM)0x4E);
  const __m512i x3 = _mm512_shuffle_epi32(x, (_MM_PERM_ENUM)0x93);
  const __m512i s = v_add(v_add(x, x1), v_add(x2, x3));
  const __m512i y = v_add(v_add(s, x), v_add(x1, x1));  // 2x_j + 3x_j+1 + x_j+2 + x_j+3
  __m512i t = v_add(y, _mm512_shuffle_i32x4(y, y, 0x4E));
  t = v_add(t, _mm512_shuffle_i32x4(t, t, 0xB1));
  return v_add(y, t);
}

BFZ_AVX512 inline __m512i v_sum16(__m512i x) {  // every lane = the sum of all 16
  __m512i h = v_add(x, _mm512_shuffle_i32x4(x, x, 0x4E));
  h = v_add(h, _mm512_shuffle_i32x4(h, h, 0xB1));
  h = v_add(h, _mm512_shuffle_epi32(h, (_MM_PERM_ENUM)0x4E));
  return v_add(h, _mm512_shuffle_epi32(h, (_MM_PERM_ENUM)0xB1));
}

BFZ_AVX512 void permute_avx512(uint32_t* s) {
  const kb::P2Tables& T = kb::P2;
  __m512i v = _mm512_loadu_si512(s);
  v = v_mds_light(v);
  for (int r = 0; r < 4; r++)
    v = v_mds_light(v_cube(v_add(v, _mm512_loadu_si512(T.ext_init[r]))));
  const __m512i dg = _mm512_loadu_si512(T.diag);
  for (int r = 0; r < 13; r++) {
    const __m512i c = v_cube(v_add(v, _mm512_maskz_set1_epi32(0x0001, (int)T.internal[r])));
    v = _mm512_mask_blend_epi32(0x0001, v, c);
    v = v_add(v_sum16(v), v_mul(v, dg));
  }
  for (int r = 0; r < 4; r++)
    v = v_mds_light(v_cube(v_add(v, _mm512_loadu_si512(T.ext_term[r]))));
  _mm512_storeu_si512(s, v);
}

// 0 = scalar, 1 = AVX-512 (checked against the scalar permutation on a few states first)
int pick() {
  if (!__builtin_cpu_supports("avx512f")) return 0;
  uint32_t a[16], b[16];
  for (int k = 0; k < 4; k++) {
    for (int i = 0; i < 16; i++) a[i] = b[i] = kb::to_mont((uint32_t)(k * 2654435761u + i * 40503u) % kb::P);
    kb::poseidon2_permute(a);
    permute_avx512(b);
    if (std::memcmp(a, b, sizeof(a)))
      throw std::runtime_error("host Poseidon2: AVX-512 permutation disagrees with the scalar one");
  }
  return 1;
}

}  // namespace

void host_permute(uint32_t s[16]) {
  static const int mode = pick();
  if (mode) permute_avx512(s);
  else kb::poseidon2_permute(s);
}

}  // namespace bfz
