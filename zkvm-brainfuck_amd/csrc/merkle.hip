// Poseidon2 Merkle tree kernels (see merkle.h).  MerkleTree::new [p3-recalled]:
//   leaf i  = sponge(row i of every tallest matrix, concatenated in commit order)
//   node j  = compress(left, right); if matrices of height == this layer exist,
//             node = compress(node, sponge(row j of those matrices))
// One thread per row/node; leaf rows are read column by column so every load of a wave is
// a contiguous 256-byte segment.
#include <algorithm>

#include "merkle.h"
#include "poseidon2.h"

// (Throughput Poseidon2 kernels at 7 or 8 waves per SIMD ran within noise of the compiler's
// 5-6: profiles/r03/ab_p2_occupancy.txt.)

namespace bfz {

using namespace kb;

// The columns hashed at one height: up to MAXSEG matrices ("segments"), segment s holding
// columns [start[s], start[s+1]) at base[s] + (c - start[s]) * stride[s].
constexpr int MAXSEG = 16;
struct ColList {
  const uint32_t* base[MAXSEG];
  size_t stride[MAXSEG];
  int start[MAXSEG + 1];
  int nseg;
  int n;
  __device__ __forceinline__ const uint32_t* col(int c) const {
    int s = 0;
    while (s + 1 < nseg && c >= start[s + 1]) s++;
    return base[s] + (size_t)(c - start[s]) * stride[s];
  }
};

__device__ __forceinline__ void sponge_cols(uint32_t st[16], const ColList& cl, size_t row) {
  for (int c0 = 0; c0 < cl.n; c0 += 8) {
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (c0 + k < cl.n) st[k] = cl.col(c0 + k)[row];
    poseidon2_permute(st);
  }
}

// Rows [r0, r0 + count) (a shard's range; the whole matrix when unsharded).
__global__ __launch_bounds__(256) void k_hash_leaves(ColList cl, size_t r0, size_t count,
                                                     uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const size_t r = r0 + i;
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
        if (cb + k < c1) st[k] = cl.col(cb + k)[j];
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

// Nodes [j0, j0 + count) of a layer.
__global__ __launch_bounds__(256) void k_compress(const uint32_t* __restrict__ prev, size_t j0,
                                                  size_t count, uint32_t* __restrict__ out,
                                                  ColList inj) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const size_t j = j0 + i;
  uint32_t st[16];
  load16(st, prev + 16 * j);
  merkle_node(st, inj, 0, inj.n, j);
  store8(out + 8 * j, st);
}

// Merkle node j in lane mode (see poseidon2_permute_lane): lane l of the node's 16-lane row
// holds word l of the state; the digest ends up in lanes 0..7.
__device__ __forceinline__ uint32_t merkle_node_lane(uint32_t v, const ColList& cl, int c0, int c1,
                                                     size_t j, int lane, const LaneConsts& kc) {
  v = poseidon2_permute_lane(v, lane, kc);
  const int nchunks = (c1 - c0 + 7) >> 3;
  if (nchunks) {
    const uint32_t d = v;
    uint32_t h = 0;
    for (int k = 0; k < nchunks; k++) {  // PaddingFreeSponge, overwrite mode
      const int col = c0 + 8 * k + lane;
      if (lane < 8 && col < c1) h = cl.col(col)[j];
      h = poseidon2_permute_lane(h, lane, kc);
    }
    const uint32_t hs = dpp<DPP_ROR8>(h);  // lanes 8..15 <- h[0..7]
    v = poseidon2_permute_lane(lane < 8 ? d : hs, lane, kc);
  }
  return v;
}

// Subtree layers in lane mode (16 lanes per node: the permutation latency, not throughput,
// is the cost here).  Block b owns TOP_NODES consecutive nodes of the first layer and
// computes their subtree up to its root: up to TOP_LAYERS layers, every layer but the first
// read from LDS, every digest written to HBM (query paths need every layer).  (A variant that
// let the last block to finish build the rest of the tree in the same launch was no faster:
// the cross-XCD release/acquire cost what the launch boundary did, profiles/r02/ab_merkle_top.txt.)
// (32- and 16-node subtrees, i.e. 512- and 256-thread blocks with one wave per SIMD from the
// first layer on, left k_compress_top's time unchanged within 3%: a layer costs one lane-mode
// permutation latency whatever the occupancy, profiles/r03/ab_open_and_tops.txt)
constexpr int TOP_NODES = 64;   // fills a 1024-thread block in one lane-mode pass
constexpr int TOP_LAYERS = 7;   // 64 nodes -> 1
// Medium layers (TOP_NODES < nodes <= LANE_LAYER_MAX) go to lane mode: a single-lane launch
// of this size is one permutation latency long (~12 us) while 16 lanes per node finish sooner.
// (2^12, 2^13, 2^15, 2^16: slower, profiles/r02/ab_merkle_top.txt, profiles/r04/ab_lane_layer_threshold.txt)
constexpr size_t LANE_LAYER_MAX = (size_t)1 << 14;
constexpr int MAXTOP = TOP_LAYERS;
struct TopLayers {
  uint32_t* out[MAXTOP];
  int c0[MAXTOP], c1[MAXTOP];
  int n;  // layers in this launch
};

// base: the first node of the launch's first layer (a rank's subtree of a sharded tree; 0 else)
__global__ __launch_bounds__(1024) void k_compress_top(const uint32_t* __restrict__ prev,
                                                       size_t nlen, ColList inj, TopLayers tl,
                                                       RootChallenge rc, size_t base) {
  __shared__ uint32_t buf[2][TOP_NODES * 8];
  const size_t per = nlen < (size_t)TOP_NODES ? nlen : (size_t)TOP_NODES;
  const size_t g0 = base + (size_t)blockIdx.x * per;  // first-layer node of this block
  const int lane = threadIdx.x & 15;
  const LaneConsts kc = lane_consts(lane);
  for (int l = 0; l < tl.n; l++) {
    const size_t m = per >> l, g = g0 >> l;
    const uint32_t* src = buf[(l - 1) & 1];
    uint32_t* dst = buf[l & 1];
    // whole 16-lane rows are active together (DPP needs all of them); the first layer is read
    // from HBM, the rest from LDS (one pointer for both would compile to flat loads)
    for (size_t j = threadIdx.x >> 4; j < m; j += blockDim.x >> 4) {
      const uint32_t x = l == 0 ? ld_global(prev, 16 * (g + j) + lane) : src[16 * j + lane];
      const uint32_t v = merkle_node_lane(x, inj, tl.c0[l], tl.c1[l], g + j, lane, kc);
      if (lane < 8) {
        tl.out[l][8 * (g + j) + lane] = v;
        dst[8 * j + lane] = v;
      }
    }
    __syncthreads();
  }
  // FRI transcript step on the finished root (the root's block only): observe the root,
  // duplex, beta = the last 4 outputs popped in reverse (as k_fri_challenge)
  if (rc.state && threadIdx.x < 64) {
    const uint32_t* root = buf[(tl.n - 1) & 1];
    uint32_t v = lane < 8 ? root[lane] : ld_global(rc.state, lane);
    v = poseidon2_permute_lane(v, lane, kc);
    if (threadIdx.x < 16) {
      rc.state[lane] = v;
      if (lane >= 4 && lane < 8) rc.beta->c[7 - lane] = v;
    }
  }
}

// Medium layers in lane mode (see LANE_LAYER_MAX).
__global__ __launch_bounds__(256) void k_compress_lanes(const uint32_t* __restrict__ prev,
                                                        size_t j0, size_t count,
                                                        uint32_t* __restrict__ out, ColList inj) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (i >= count) return;
  const size_t j = j0 + i;
  const uint32_t v = merkle_node_lane(prev[16 * j + lane], inj, 0, inj.n, j, lane, lane_consts(lane));
  if (lane < 8) out[8 * j + lane] = v;
}

__global__ __launch_bounds__(256) void k_hash_rows8_lanes(const uint32_t* __restrict__ rows,
                                                          size_t r0, size_t count,
                                                          uint32_t* __restrict__ out) {
  const size_t i = r0 + (((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4);
  const int lane = threadIdx.x & 15;
  if (i >= r0 + count) return;
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

__global__ __launch_bounds__(256) void k_hash_rows8(const uint32_t* __restrict__ rows, size_t r0,
                                                    size_t count, uint32_t* __restrict__ out) {
  const size_t i = r0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= r0 + count) return;
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
  cl.nseg = 0;
  for (const MatRef* m : ms) {
    if (cl.nseg >= MAXSEG) throw std::runtime_error("merkle: too many matrices at one height");
    cl.base[cl.nseg] = m->base;
    cl.stride[cl.nseg] = m->stride ? m->stride : m->height;
    cl.start[cl.nseg] = cl.n;
    cl.nseg++;
    cl.n += m->width;
  }
  cl.start[cl.nseg] = cl.n;
  return cl;
}

// One layer's nodes [j0, j0 + count) from layers[L-1] (lane mode for small launches).
static void launch_layer(MerkleTree& t, int L, size_t j0, size_t count,
                         const std::vector<const MatRef*>& grp, hipStream_t st) {
  const uint32_t* prev = t.layers[L - 1].p;
  if (count <= LANE_LAYER_MAX)
    hipLaunchKernelGGL(k_compress_lanes, dim3(ceil_div(16 * count, 256)), dim3(256), 0, st, prev,
                       j0, count, t.layers[L].p, make_cols(grp));
  else {
    const ColList cl = make_cols(grp);
    KernelProbe& probe = p2_probe();
    hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
    hipLaunchKernelGGL(k_compress, dim3(ceil_div(count, 256)), dim3(256), 0, st, prev, j0, count,
                       t.layers[L].p, cl);
    // one compression, plus the injected rows' sponge and one more compression if any
    if (probe.on)
      probe.end(ev0, st, (double)count * (cl.n ? 2 + (cl.n + 7) / 8 : 1), cl.n ? "k_compress+inject" : "k_compress");
  }
  KCHECK();
}

// Layers L0..nl with layers[L0-1] (len nodes) complete; sorted[next..] are the matrices
// still to inject (heights descending).  Big layers get one launch each; the rest go to
// k_compress_top in one launch.
static void build_layers(MerkleTree& t, int L0, size_t len, const std::vector<const MatRef*>& sorted,
                         size_t next, hipStream_t st, bool fetch_root = true,
                         RootChallenge rc = {}) {
  const int nl = (int)t.layers.size() - 1;
  int L = L0;
  for (; L <= nl && (len >> 1) > LANE_LAYER_MAX; L++) {  // throughput layers
    const size_t nlen = len >> 1;
    std::vector<const MatRef*> grp;
    while (next < sorted.size() && sorted[next]->height == nlen) grp.push_back(sorted[next++]);
    t.layers[L].reset(8 * nlen);
    launch_layer(t, L, 0, nlen, grp, st);
    len = nlen;
  }
  while (L <= nl) {  // subtree launches
    const size_t first = len >> 1;
    const int sub = first > (size_t)TOP_NODES ? TOP_LAYERS : log2i(first) + 1;
    TopLayers tl{};
    tl.n = std::min(sub, nl - L + 1);
    std::vector<const MatRef*> all;
    size_t nlen = first;
    for (int l = 0; l < tl.n; l++, nlen >>= 1) {
      tl.c0[l] = 0;
      for (const MatRef* m : all) tl.c0[l] += m->width;
      while (next < sorted.size() && sorted[next]->height == nlen) all.push_back(sorted[next++]);
      tl.c1[l] = 0;
      for (const MatRef* m : all) tl.c1[l] += m->width;
      t.layers[L + l].reset(8 * nlen);
      tl.out[l] = t.layers[L + l].p;
    }
    const unsigned blocks = first > (size_t)TOP_NODES ? (unsigned)(first / TOP_NODES) : 1u;
    const bool root_launch = L + tl.n > nl;
    hipLaunchKernelGGL(k_compress_top, dim3(blocks), dim3(16 * TOP_NODES), 0, st,
                       (const uint32_t*)t.layers[L - 1].p, first, make_cols(all), tl,
                       root_launch ? rc : RootChallenge{}, (size_t)0);
    KCHECK();
    L += tl.n;
    len = first >> (tl.n - 1);
  }
  if (next != sorted.size()) throw std::runtime_error("merkle: non power-of-two heights");
  if (!fetch_root) return;
  fetch(t.root, t.layers[nl].p, 32, st);
}

// ------------------------------------------------------------------ sharded trees
ShardCtx*& shard_ctx() {
  static ShardCtx* c = nullptr;
  return c;
}

static bool shard_tree(size_t h0) {
  const ShardCtx* c = shard_ctx();
  return c && c->world > 1 && h0 >= (size_t)c->world * SHARD_MIN_LEAVES;
}

// Rank k owns nodes [k len / G, (k+1) len / G) of every layer with len >= G nodes (one
// subtree, injected rows included); the layer of G nodes is all-gathered and the layers above
// it are built redundantly by every rank.  leaves(r0, count) hashes the rank's own rows.
template <class Leaves>
static void build_sharded(MerkleTree& t, size_t h0, const std::vector<const MatRef*>& sorted,
                          size_t next, Leaves leaves, hipStream_t st, bool fetch_root,
                          RootChallenge rc = {}) {
  const ShardCtx& c = *shard_ctx();
  const size_t G = (size_t)c.world, k = (size_t)c.rank;
  const int nl = log2i(h0), lg = log2i(G);
  t.sharded_below = nl - lg;  // layers [0, nl - lg) hold only this rank's range
  t.shard_log = lg;
  leaves(k * (h0 / G), h0 / G);
  size_t len = h0;
  int L = 1;
  for (; L <= nl - lg && (len >> 1) / G > LANE_LAYER_MAX; L++) {  // throughput layers
    const size_t nlen = len >> 1;
    std::vector<const MatRef*> grp;
    while (next < sorted.size() && sorted[next]->height == nlen) grp.push_back(sorted[next++]);
    t.layers[L].reset(8 * nlen);
    launch_layer(t, L, k * (nlen / G), nlen / G, grp, st);
    len = nlen;
  }
  // the rank's subtree below the shard level: up to TOP_LAYERS layers per k_compress_top launch
  // (a layer per launch made the small shares of a many-rank proof launch-bound)
  while (L <= nl - lg) {
    const size_t first = (len >> 1) / G;  // this rank's nodes of the launch's first layer
    const int sub = first > (size_t)TOP_NODES ? TOP_LAYERS : log2i(first) + 1;
    TopLayers tl{};
    tl.n = std::min(sub, nl - lg - L + 1);
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
    const unsigned blocks = first > (size_t)TOP_NODES ? (unsigned)(first / TOP_NODES) : 1u;
    hipLaunchKernelGGL(k_compress_top, dim3(blocks), dim3(16 * TOP_NODES), 0, st,
                       (const uint32_t*)t.layers[L - 1].p, first, make_cols(all), tl,
                       RootChallenge{}, k * first);
    KCHECK();
    L += tl.n;
    len >>= tl.n;
  }
  // layer nl - lg has G nodes; node k is ours: all-gather them device to device
  DBuf<uint32_t>& lay = t.layers[nl - lg];
  DBuf<uint32_t> all(8 * G);
  coll_sync(st);
  c.allgather(lay.p + 8 * k, 32, all.p);
  HIP_CHECK(hipMemcpyAsync(lay.p, all.p, 32 * G, hipMemcpyDeviceToDevice, st));
  build_layers(t, nl - lg + 1, G, sorted, next, st, fetch_root, rc);
}

void merkle_build(const std::vector<MatRef>& mats, MerkleTree& t, hipStream_t st, bool fetch_root) {
  if (mats.empty()) throw std::runtime_error("merkle: no matrices");
  t.mats = mats;
  std::vector<const MatRef*> sorted;
  for (const MatRef& m : mats) sorted.push_back(&m);
  std::stable_sort(sorted.begin(), sorted.end(),
                   [](const MatRef* a, const MatRef* b) { return a->height > b->height; });
  const size_t h0 = sorted[0]->height;
  t.layers.clear();
  t.layers.resize(log2i(h0) + 1);
  t.sharded_below = 0;
  size_t next = 0;
  std::vector<const MatRef*> grp;
  while (next < sorted.size() && sorted[next]->height == h0) grp.push_back(sorted[next++]);
  t.layers[0].reset(8 * h0);
  const ColList cl = make_cols(grp);
  auto leaves = [&](size_t r0, size_t count) {
    KernelProbe& probe = p2_probe();
    hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
    hipLaunchKernelGGL(k_hash_leaves, dim3(ceil_div(count, 256)), dim3(256), 0, st, cl, r0,
                       count, t.layers[0].p);
    KCHECK();
    if (probe.on) probe.end(ev0, st, (double)count * ((cl.n + 7) / 8), "k_hash_leaves");
  };
  if (shard_tree(h0)) {
    build_sharded(t, h0, sorted, next, leaves, st, fetch_root);
    return;
  }
  leaves(0, h0);
  build_layers(t, 1, h0, sorted, next, st, fetch_root);
}

static void hash_rows8_range(const uint32_t* rows, size_t r0, size_t count, uint32_t* digests,
                             hipStream_t st) {
  if (count <= LANE_LAYER_MAX)
    hipLaunchKernelGGL(k_hash_rows8_lanes, dim3(ceil_div(16 * count, 256)), dim3(256), 0, st, rows,
                       r0, count, digests);
  else {
    KernelProbe& probe = p2_probe();
    hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
    hipLaunchKernelGGL(k_hash_rows8, dim3(ceil_div(count, 256)), dim3(256), 0, st, rows, r0, count,
                       digests);
    if (probe.on) probe.end(ev0, st, (double)count, "k_hash_rows8");
  }
  KCHECK();
}

void merkle_from_rows8(MerkleTree& t, const uint32_t* rows, size_t h, hipStream_t st,
                       bool fetch_root, RootChallenge rc, bool allow_shard,
                       const std::function<void(size_t, size_t, uint32_t*)>& fused) {
  t.mats = {MatRef{rows, h, 8}};
  t.layers.clear();
  t.layers.resize(log2i(h) + 1);
  t.layers[0].reset(8 * h);
  t.sharded_below = 0;
  auto leaves = [&](size_t r0, size_t count) {
    if (fused) fused(r0, count, t.layers[0].p);
    else hash_rows8_range(rows, r0, count, t.layers[0].p, st);
  };
  if (h < 2) throw std::runtime_error("merkle: rows8 tree needs two leaves");
  if (allow_shard && shard_tree(h)) {
    build_sharded(t, h, {}, 0, leaves, st, fetch_root, rc);
    return;
  }
  leaves(0, h);
  build_layers(t, 1, h, {}, 0, st, fetch_root, rc);
}

void poseidon2_batch(uint32_t* states, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_permute_batch, dim3(ceil_div(n, 256)), dim3(256), 0, st, states, n);
  KCHECK();
}

void poseidon2_batch_small(uint32_t* states, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_permute_lanes, dim3(ceil_div(16 * n, 256)), dim3(256), 0, st, states, n);
  KCHECK();
}

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_merkle{
    (const void*)&k_hash_leaves,
    (const void*)&k_compress,
    (const void*)&k_compress_top,
    (const void*)&k_compress_lanes,
    (const void*)&k_hash_rows8_lanes,
    (const void*)&k_hash_rows8};

}  // namespace bfz
