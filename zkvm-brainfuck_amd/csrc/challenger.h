// The prover's DuplexChallenger (prover.hip: Challenger; p3 DuplexChallenger, decision D7) on the
// device, for the transcript steps that run there so the GPU does not wait for the host: one
// 16-lane row holds the sponge (lane l: state word l; lanes 0..7 the input and output buffers;
// nin / nout uniform).  The host replays every step when the roots come back.
#pragma once
#include "poseidon2.h"

namespace bfz {

struct DevChallenger {  // the host Challenger's fields, in device memory
  uint32_t st[16];
  uint32_t in[8];
  int32_t nin;
  uint32_t out[8];
  int32_t nout;
};

#ifdef __HIPCC__
struct LaneSponge {
  int lane;
  kb::LaneConsts kc;
  uint32_t stv, inv, outv;
  int nin, nout;
  __device__ void load(const DevChallenger* c) {
    lane = threadIdx.x & 15;
    kc = kb::lane_consts(lane);
    stv = c->st[lane];
    inv = lane < 8 ? c->in[lane] : 0u;
    outv = lane < 8 ? c->out[lane] : 0u;
    nin = c->nin;
    nout = c->nout;
  }
  // threads 0..15 (row 0) write the state back
  __device__ void store(DevChallenger* c) const {
    if (threadIdx.x >= 16) return;
    c->st[lane] = stv;
    if (lane < 8) {
      c->in[lane] = inv;
      c->out[lane] = outv;
    }
    if (lane == 0) {
      c->nin = nin;
      c->nout = nout;
    }
  }
  __device__ void duplex() {
    if (lane < nin) stv = inv;
    stv = kb::poseidon2_permute_lane(stv, lane, kc);
    outv = stv;
    nout = 8;
    nin = 0;
  }
  __device__ void observe(uint32_t v) {
    nout = 0;
    if (lane == nin) inv = v;
    if (++nin == 8) duplex();
  }
  __device__ uint32_t sample() {
    if (nin > 0 || nout == 0) duplex();
    --nout;
    return (uint32_t)__shfl(outv, nout, 16);
  }
  __device__ kb::EF sample_ef() {
    kb::EF r;
    for (int e = 0; e < 4; e++) r.c[e] = sample();
    return r;
  }
};
#endif

}  // namespace bfz
