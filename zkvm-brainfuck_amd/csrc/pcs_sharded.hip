// Column-sharded PCS commit + FRI commit phase.
//
//   1. coset LDE of the rank's columns (n -> 2n, shift GENERATOR = 3, bit-reversed rows), as
//      Pcs::commit does per matrix (prover.rs:209-236);
//   2. one all-to-all turns column shards into row shards: block j of every local column goes
//      to rank j, so rank k receives rows [k 2n/G, (k+1) 2n/G) of all w columns, column-major
//      (the receive buffer needs no unpacking);
//   3. MerkleTreeMmcs commit: rank k hashes its rows and builds its subtree; the G subtree roots
//      are all-gathered and the top log2 G layers are built by every rank (merkle.hip);
//   4. FRI input: f(x) = sum_c alpha^c col_c(x) at the rank's rows, alpha sampled from the
//      DuplexChallenger after observing the root (the batching step of the reduced opening);
//   5. FRI commit phase (fri::prover::commit_phase): per round, commit pairs of EF values
//      (one permutation per leaf), observe the root, sample beta, fold.  Rounds stay row
//      sharded while a layer has >= G * 1024 leaves; the first smaller layer is all-gathered
//      (at most 2 G * 1024 EF values) and the rest runs redundantly on every rank.
// Every rank returns the same roots and final value, equal to the world = 1 run: the synthetic
// trace is a polynomial of degree < n, so the fold must end in a constant (checked).
#include "pcs_sharded.h"

#include <stdexcept>

#include "fri.h"
#include "merkle.h"
#include "ntt.h"

namespace bfz {

using namespace kb;

// out[i] = sum_c apow[c] * col_c[i]   (lazy 64-bit dot product, kb::LazyEF)
__global__ __launch_bounds__(256) void k_lincomb(const uint32_t* __restrict__ cols, size_t stride,
                                                 int w, size_t count,
                                                 const EF* __restrict__ apow,
                                                 EF* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  LazyEF lz;
  lz.init();
  for (int c = 0; c < w; c++) lz.add(apow[c], cols[(size_t)c * stride + i]);
  out[i] = lz.get();
}

PcsShardedResult commit_fri_sharded(const uint32_t* cols, int log_n, int w_local, uint32_t* send,
                                    uint32_t* recv, const std::function<void()>& alltoall,
                                    hipStream_t st) {
  const ShardCtx* sc = shard_ctx();
  const int G = sc && sc->world > 1 ? sc->world : 1, k = G > 1 ? sc->rank : 0;
  const size_t n = (size_t)1 << log_n, H = 2 * n, blk = H / G;
  if (w_local < 1) throw std::runtime_error("pcs: no columns");
  if (G > 1 && blk < SHARD_MIN_LEAVES) throw std::runtime_error("pcs: 2n / world < 1024 rows");
  if (G > 1 && (!send || !recv)) throw std::runtime_error("pcs: exchange buffers missing");

  // 1. LDE of the local columns
  DBuf<uint32_t> lde(H * (size_t)w_local);
  coset_lde(cols, n, w_local, to_mont(3), lde.p, st);

  // 2. column shards -> row shards
  const uint32_t* rows = lde.p;
  size_t rstride = H;
  if (G > 1) {
    for (int j = 0; j < G; j++)
      HIP_CHECK(hipMemcpy2DAsync(send + (size_t)j * w_local * blk, blk * 4, lde.p + (size_t)j * blk,
                                 H * 4, blk * 4, w_local, hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
    alltoall();
    rows = recv;
    rstride = blk;
  }
  const int W = w_local * G;

  // 3. commit: one matrix whose row r of column c sits at rows[c * rstride + r - k * blk]
  //    (only the rank's rows are read)
  PcsShardedResult res;
  {
    std::vector<MatRef> mats{MatRef{rows - (size_t)k * blk, H, W, rstride}};
    MerkleTree tree;
    merkle_build(mats, tree, st);
    std::copy(tree.root, tree.root + 8, res.root);
  }

  // 4. FRI input
  Challenger ch;
  ch.observe_digest(res.root);
  const EF alpha = ch.sample_ef();
  std::vector<EF> ap(W);
  ap[0] = ef_one();
  for (int c = 1; c < W; c++) ap[c] = ef_mul(ap[c - 1], alpha);
  DBuf<EF> dap(W);
  HIP_CHECK(hipMemcpyAsync(dap.p, ap.data(), W * sizeof(EF), hipMemcpyHostToDevice, st));
  bool local = G > 1;
  DBuf<EF> cur(local ? blk : H);
  hipLaunchKernelGGL(k_lincomb, dim3(ceil_div(cur.n, 256)), dim3(256), 0, st, rows, rstride, W,
                     cur.n, (const EF*)dap.p, cur.p);
  KCHECK();
  HIP_CHECK(hipStreamSynchronize(st));  // ap, dap stay valid until here

  // 5. commit phase: the transcript step runs on the device (observe root, duplex, beta)
  DBuf<uint32_t> dstate(16);
  HIP_CHECK(hipMemcpyAsync(dstate.p, ch.st, 64, hipMemcpyHostToDevice, st));
  DBuf<EF> betas(log2i(H));
  std::vector<MerkleTree> trees;
  size_t len = H;
  for (int rd = 0; len > 2; rd++) {
    const size_t h = len / 2;
    if (local && h < (size_t)G * SHARD_MIN_LEAVES) {  // gather the layer, finish redundantly
      DBuf<EF> all(len);  // device to device
      HIP_CHECK(hipStreamSynchronize(st));
      sc->allgather(cur.p, (len / G) * sizeof(EF), all.p);
      cur = std::move(all);
      local = false;
    }
    const size_t i0 = local ? (size_t)k * (h / G) : 0, cnt = local ? h / G : h;
    trees.emplace_back();
    MerkleTree& t = trees.back();
    merkle_from_rows8(t, reinterpret_cast<const uint32_t*>(cur.p) - 8 * i0, h, st, false,
                      RootChallenge{dstate.p, betas.p + rd});
    DBuf<EF> next(cnt);
    fri_fold_range(cur.p, next.p, h, i0, cnt, betas.p + rd, nullptr, st);
    cur = std::move(next);
    len = h;
  }
  res.fri_roots.resize(trees.size());
  for (size_t i = 0; i < trees.size(); i++)
    HIP_CHECK(hipMemcpyAsync(res.fri_roots[i].data(), trees[i].layers.back().p, 32,
                             hipMemcpyDeviceToHost, st));
  EF fin[2];
  HIP_CHECK(hipMemcpyAsync(fin, cur.p, sizeof(fin), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  if (!ef_eq(fin[0], fin[1])) throw std::runtime_error("pcs: FRI did not fold to a constant");
  res.final_value = fin[0];
  return res;
}

}  // namespace bfz
