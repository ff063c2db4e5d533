// Poseidon2 Merkle tree kernels (see merkle.h).  MerkleTree::new [p3-recalled]:
//   leaf i  = sponge(row i of every tallest matrix, concatenated in commit order)
//   node j  = compress(left, right); if matrices of height == this layer exist,
//             node = compress(node, sponge(row j of those matrices))
// One thread per row/node; leaf rows are read column by column so every load of a wave is
// a contiguous 256-byte segment.
#include <algorithm>

#include "merkle.h"
#include "poseidon2.h"

namespace bfz {

using namespace kb;

constexpr int MAXCOLS = 160;
struct ColList {
  const uint32_t* p[MAXCOLS];
  int n;
};

__device__ __forceinline__ void sponge_cols(uint32_t st[16], const ColList& cl, size_t row) {
  for (int c0 = 0; c0 < cl.n; c0 += 8) {
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (c0 + k < cl.n) st[k] = cl.p[c0 + k][row];
    poseidon2_permute(st);
  }
}

__global__ __launch_bounds__(256) void k_hash_leaves(ColList cl, size_t height,
                                                     uint32_t* __restrict__ out) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= height) return;
  uint32_t st[16];
#pragma unroll
  for (int i = 0; i < 16; i++) st[i] = 0;
  sponge_cols(st, cl, r);
  uint4* o = reinterpret_cast<uint4*>(out + 8 * r);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

// Merkle node j from its two children already in st[0..16]:
//   compress(children), then with injected columns [c0, c1): compress(node, sponge(row j)).
// The steps share ONE permutation call site, so the kernel holds a single inlined copy of
// the (~37 KB) permutation instead of three.
__device__ __forceinline__ void merkle_node(uint32_t st[16], const ColList& cl, int c0, int c1,
                                            size_t j) {
  const int nchunks = (c1 - c0 + 7) >> 3;
  const int nsteps = nchunks ? nchunks + 2 : 1;
  uint32_t d[8];
  for (int step = 0; step < nsteps; step++) {
    if (step == 1) {
#pragma unroll
      for (int i = 0; i < 8; i++) d[i] = st[i];
#pragma unroll
      for (int i = 0; i < 16; i++) st[i] = 0;
    }
    if (step >= 1 && step <= nchunks) {
      const int cb = c0 + 8 * (step - 1);
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (cb + k < c1) st[k] = cl.p[cb + k][j];
    }
    if (nchunks && step == nchunks + 1) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        st[8 + i] = st[i];
        st[i] = d[i];
      }
    }
    poseidon2_permute(st);
  }
}

__device__ __forceinline__ void load16(uint32_t st[16], const uint32_t* p) {
  const uint4* in = reinterpret_cast<const uint4*>(p);
  const uint4 a = in[0], b = in[1], c = in[2], d = in[3];
  st[0] = a.x; st[1] = a.y; st[2] = a.z; st[3] = a.w;
  st[4] = b.x; st[5] = b.y; st[6] = b.z; st[7] = b.w;
  st[8] = c.x; st[9] = c.y; st[10] = c.z; st[11] = c.w;
  st[12] = d.x; st[13] = d.y; st[14] = d.z; st[15] = d.w;
}

__device__ __forceinline__ void store8(uint32_t* p, const uint32_t st[16]) {
  uint4* o = reinterpret_cast<uint4*>(p);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

__global__ __launch_bounds__(256) void k_compress(const uint32_t* __restrict__ prev, size_t nlen,
                                                  uint32_t* __restrict__ out, ColList inj) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nlen) return;
  uint32_t st[16];
  load16(st, prev + 16 * j);
  merkle_node(st, inj, 0, inj.n, j);
  store8(out + 8 * j, st);
}

// Merkle node j in lane mode (see poseidon2_permute_lane): lane l of the node's 16-lane row
// holds word l of the state; the digest ends up in lanes 0..7.
__device__ __forceinline__ uint32_t merkle_node_lane(uint32_t v, const ColList& cl, int c0, int c1,
                                                     size_t j, int lane) {
  v = poseidon2_permute_lane(v, lane);
  const int nchunks = (c1 - c0 + 7) >> 3;
  if (nchunks) {
    const uint32_t d = v;
    uint32_t h = 0;
    for (int k = 0; k < nchunks; k++) {  // PaddingFreeSponge, overwrite mode
      const int col = c0 + 8 * k + lane;
      if (lane < 8 && col < c1) h = cl.p[col][j];
      h = poseidon2_permute_lane(h, lane);
    }
    const uint32_t hs = dpp<DPP_ROR8>(h);  // lanes 8..15 <- h[0..7]
    v = poseidon2_permute_lane(lane < 8 ? d : hs, lane);
  }
  return v;
}

// All layers of <= TOP_NODES nodes in one workgroup: layer l reads the previous layer from
// LDS (the first from HBM), writes its digests to HBM (query paths need every layer) and to
// LDS for the next.  Layers of <= LANE_NODES nodes switch to lane mode (16 lanes per node):
// there the permutation latency, not throughput, is the cost.
constexpr int TOP_NODES = 512;
constexpr int LANE_NODES = 256;   // up to 4 batches of 64 nodes per 1024-thread block
constexpr int MAXTOP = 24;
struct TopLayers {
  uint32_t* out[MAXTOP];
  int c0[MAXTOP], c1[MAXTOP];
  int n;
};

__global__ __launch_bounds__(1024) void k_compress_top(const uint32_t* __restrict__ prev,
                                                       size_t nlen, ColList inj, TopLayers tl) {
  __shared__ uint4 buf[2][TOP_NODES * 2];
  for (int l = 0; l < tl.n; l++, nlen >>= 1) {
    const uint32_t* src32 = l == 0 ? prev : reinterpret_cast<const uint32_t*>(buf[(l - 1) & 1]);
    uint32_t* dst32 = reinterpret_cast<uint32_t*>(buf[l & 1]);
    if (nlen <= (size_t)LANE_NODES) {
      const int lane = threadIdx.x & 15;
      for (size_t j = threadIdx.x >> 4; j < nlen; j += blockDim.x >> 4) {
        // whole 16-lane rows are active together (DPP needs all of them)
        const uint32_t v = merkle_node_lane(src32[16 * j + lane], inj, tl.c0[l], tl.c1[l], j, lane);
        if (lane < 8) {
          tl.out[l][8 * j + lane] = v;
          dst32[8 * j + lane] = v;
        }
      }
    } else {
      for (size_t j = threadIdx.x; j < nlen; j += blockDim.x) {
        uint32_t st[16];
        if (l == 0) {
          load16(st, prev + 16 * j);
        } else {
          const uint4* s4 = buf[(l - 1) & 1] + 4 * j;
          const uint4 a = s4[0], b = s4[1], c = s4[2], d = s4[3];
          st[0] = a.x; st[1] = a.y; st[2] = a.z; st[3] = a.w;
          st[4] = b.x; st[5] = b.y; st[6] = b.z; st[7] = b.w;
          st[8] = c.x; st[9] = c.y; st[10] = c.z; st[11] = c.w;
          st[12] = d.x; st[13] = d.y; st[14] = d.z; st[15] = d.w;
        }
        merkle_node(st, inj, tl.c0[l], tl.c1[l], j);
        store8(tl.out[l] + 8 * j, st);
        buf[l & 1][2 * j] = make_uint4(st[0], st[1], st[2], st[3]);
        buf[l & 1][2 * j + 1] = make_uint4(st[4], st[5], st[6], st[7]);
      }
    }
    __syncthreads();
  }
}

// Medium layers (TOP_NODES < nodes <= LANE_LAYER_MAX) in lane mode: a single-lane launch of
// this size is one permutation latency long (~12 us) while 16 lanes per node finish sooner.
constexpr size_t LANE_LAYER_MAX = (size_t)1 << 14;
__global__ __launch_bounds__(256) void k_compress_lanes(const uint32_t* __restrict__ prev,
                                                        size_t nlen, uint32_t* __restrict__ out,
                                                        ColList inj) {
  const size_t j = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (j >= nlen) return;
  const uint32_t v = merkle_node_lane(prev[16 * j + lane], inj, 0, inj.n, j, lane);
  if (lane < 8) out[8 * j + lane] = v;
}

__global__ __launch_bounds__(256) void k_hash_rows8_lanes(const uint32_t* __restrict__ rows,
                                                          size_t n, uint32_t* __restrict__ out) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (i >= n) return;
  const uint32_t v = poseidon2_permute_lane(lane < 8 ? rows[8 * i + lane] : 0u, lane);
  if (lane < 8) out[8 * i + lane] = v;
}

// Lane-mode batch permutation (bfz_poseidon2_permute_small): 16 lanes per state.
__global__ __launch_bounds__(256) void k_permute_lanes(uint32_t* __restrict__ s, size_t n) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (i >= n) return;
  s[16 * i + lane] = poseidon2_permute_lane(s[16 * i + lane], lane);
}

__global__ __launch_bounds__(256) void k_permute_batch(uint32_t* __restrict__ s, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t st[16];
#pragma unroll
  for (int k = 0; k < 16; k++) st[k] = s[16 * i + k];
  poseidon2_permute(st);
#pragma unroll
  for (int k = 0; k < 16; k++) s[16 * i + k] = st[k];
}

__global__ __launch_bounds__(256) void k_hash_rows8(const uint32_t* __restrict__ rows, size_t n,
                                                    uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t st[16];
  const uint4* in = reinterpret_cast<const uint4*>(rows + 8 * i);
  uint4 a = in[0], b = in[1];
  st[0] = a.x; st[1] = a.y; st[2] = a.z; st[3] = a.w;
  st[4] = b.x; st[5] = b.y; st[6] = b.z; st[7] = b.w;
#pragma unroll
  for (int k = 8; k < 16; k++) st[k] = 0;
  poseidon2_permute(st);
  uint4* o = reinterpret_cast<uint4*>(out + 8 * i);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

static ColList make_cols(const std::vector<const MatRef*>& ms) {
  ColList cl{};
  cl.n = 0;
  for (const MatRef* m : ms)
    for (int c = 0; c < m->width; c++) {
      if (cl.n >= MAXCOLS) throw std::runtime_error("merkle: too many columns at one height");
      cl.p[cl.n++] = m->base + (size_t)c * m->height;
    }
  return cl;
}

// Layers 1..nl above layers[0]; sorted[next..] are the matrices still to inject (heights
// descending).  Big layers get one launch each; the rest go to k_compress_top in one launch.
static void build_layers(MerkleTree& t, size_t len, const std::vector<const MatRef*>& sorted,
                         size_t next, hipStream_t st, bool fetch_root = true) {
  const int nl = log2i(len);
  int L = 1;
  for (; L <= nl && (len >> 1) > (size_t)TOP_NODES; L++) {
    const size_t nlen = len >> 1;
    std::vector<const MatRef*> grp;
    while (next < sorted.size() && sorted[next]->height == nlen) grp.push_back(sorted[next++]);
    t.layers[L].reset(8 * nlen);
    if (nlen <= LANE_LAYER_MAX)
      hipLaunchKernelGGL(k_compress_lanes, dim3(ceil_div(16 * nlen, 256)), dim3(256), 0, st,
                         (const uint32_t*)t.layers[L - 1].p, nlen, t.layers[L].p, make_cols(grp));
    else
      hipLaunchKernelGGL(k_compress, dim3(ceil_div(nlen, 256)), dim3(256), 0, st,
                         (const uint32_t*)t.layers[L - 1].p, nlen, t.layers[L].p, make_cols(grp));
    KCHECK();
    len = nlen;
  }
  if (L <= nl) {
    TopLayers tl{};
    tl.n = nl - L + 1;
    if (tl.n > MAXTOP) throw std::runtime_error("merkle: too many top layers");
    std::vector<const MatRef*> all;
    size_t nlen = len >> 1;
    for (int l = 0; l < tl.n; l++, nlen >>= 1) {
      tl.c0[l] = 0;
      for (const MatRef* m : all) tl.c0[l] += m->width;
      while (next < sorted.size() && sorted[next]->height == nlen) all.push_back(sorted[next++]);
      tl.c1[l] = 0;
      for (const MatRef* m : all) tl.c1[l] += m->width;
      t.layers[L + l].reset(8 * nlen);
      tl.out[l] = t.layers[L + l].p;
    }
    hipLaunchKernelGGL(k_compress_top, dim3(1), dim3(1024), 0, st,
                       (const uint32_t*)t.layers[L - 1].p, len >> 1, make_cols(all), tl);
    KCHECK();
  }
  if (next != sorted.size()) throw std::runtime_error("merkle: non power-of-two heights");
  if (!fetch_root) return;
  HIP_CHECK(hipMemcpyAsync(t.root, t.layers[nl].p, 32, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
}

void merkle_build(const std::vector<MatRef>& mats, MerkleTree& t, hipStream_t st) {
  if (mats.empty()) throw std::runtime_error("merkle: no matrices");
  t.mats = mats;
  std::vector<const MatRef*> sorted;
  for (const MatRef& m : mats) sorted.push_back(&m);
  std::stable_sort(sorted.begin(), sorted.end(),
                   [](const MatRef* a, const MatRef* b) { return a->height > b->height; });
  const size_t h0 = sorted[0]->height;
  t.layers.clear();
  t.layers.resize(log2i(h0) + 1);
  size_t next = 0;
  std::vector<const MatRef*> grp;
  while (next < sorted.size() && sorted[next]->height == h0) grp.push_back(sorted[next++]);
  t.layers[0].reset(8 * h0);
  hipLaunchKernelGGL(k_hash_leaves, dim3(ceil_div(h0, 256)), dim3(256), 0, st, make_cols(grp), h0,
                     t.layers[0].p);
  KCHECK();
  build_layers(t, h0, sorted, next, st);
}

void merkle_layers_from_leaves(MerkleTree& t, hipStream_t st, bool fetch_root) {
  const size_t len = t.mats.empty() ? 0 : t.mats[0].height;
  t.layers.resize(log2i(len) + 1);
  build_layers(t, len, {}, 0, st, fetch_root);
}

void poseidon2_batch(uint32_t* states, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_permute_batch, dim3(ceil_div(n, 256)), dim3(256), 0, st, states, n);
  KCHECK();
}

void poseidon2_batch_small(uint32_t* states, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_permute_lanes, dim3(ceil_div(16 * n, 256)), dim3(256), 0, st, states, n);
  KCHECK();
}

void hash_rows8(const uint32_t* rows, size_t n, uint32_t* digests, hipStream_t st) {
  if (n <= LANE_LAYER_MAX)
    hipLaunchKernelGGL(k_hash_rows8_lanes, dim3(ceil_div(16 * n, 256)), dim3(256), 0, st, rows, n,
                       digests);
  else
    hipLaunchKernelGGL(k_hash_rows8, dim3(ceil_div(n, 256)), dim3(256), 0, st, rows, n, digests);
  KCHECK();
}

}  // namespace bfz
