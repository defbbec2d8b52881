// Cross-entropy over the (padded) vocabulary with the gradient written in place.
//
// Reference: F.cross_entropy on shifted [B*(S-1), V] logits, fp32 under autocast
// (gpt.py:449-453; SURVEY §2.5 K11/K12: the fp32 log_softmax alone is 1.65 GB for
// small at B=8).  Here the bf16 logits buffer [M, Vp] from the lm_head GEMM is
// read twice (online max/sum pass, then grad pass) and overwritten by
//   dlogits = (softmax(l) - onehot(target)) / n_valid       (0 for padded columns
// and for rows whose target is ignore_index), so no fp32 logits or separate
// softmax-backward kernel ever exist.  One 256-thread block per row; loads are 16 B.
#include "common.h"

__global__ __launch_bounds__(256) void k_ce_fwd_bwd(bf16_t* __restrict__ logits, const int64_t* __restrict__ targets,
                                                    const int64_t* __restrict__ n_valid, float* __restrict__ loss_rows,
                                                    int M, int Vp, int V) {
  __shared__ float sm_m[4], sm_s[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  bf16_t* lrow = logits + (size_t)row * Vp;
  const int64_t tgt = targets[row];
  const bool valid = tgt >= 0 && tgt < V;
  const int nchunk = Vp >> 3;
  // pass 1: online max / sum-exp
  float mx = -INFINITY, sm = 0.f;
  for (int c = tid; c < nchunk; c += 256) {
    const u16x8 x = *reinterpret_cast<const u16x8*>(lrow + c * 8);
    float v[8];
    float lm = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = (c * 8 + e < V) ? bf2f(x.v[e]) : -INFINITY;
      lm = fmaxf(lm, v[e]);
    }
    if (lm > mx) { sm *= __expf(mx - lm); mx = lm; }
    if (mx != -INFINITY) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sm += __expf(v[e] - mx);
    }
  }
  // wave reduce (max, sum) pairs
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64), os = __shfl_xor(sm, o, 64);
    const float nm = fmaxf(mx, om);
    sm = (mx == -INFINITY ? 0.f : sm * __expf(mx - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    mx = nm;
  }
  if (lane == 0) { sm_m[wid] = mx; sm_s[wid] = sm; }
  __syncthreads();
  float gm = fmaxf(fmaxf(sm_m[0], sm_m[1]), fmaxf(sm_m[2], sm_m[3]));
  float gs = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) gs += (sm_m[w] == -INFINITY) ? 0.f : sm_s[w] * __expf(sm_m[w] - gm);
  const float lse = gm + __logf(gs);
  if (tid == 0) loss_rows[row] = valid ? (lse - bf2f(lrow[tgt])) : 0.f;
  __syncthreads();  // everyone has read lrow[tgt] before it is overwritten
  const int64_t nv = *n_valid;
  const float inv_n = valid ? 1.f / (float)(nv > 0 ? nv : 1) : 0.f;
  // pass 2: gradient in place
  for (int c = tid; c < nchunk; c += 256) {
    u16x8 x = *reinterpret_cast<const u16x8*>(lrow + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = c * 8 + e;
      float g = 0.f;
      if (col < V) {
        g = __expf(bf2f(x.v[e]) - lse);
        if (col == tgt) g -= 1.f;
        g *= inv_n;
      }
      x.v[e] = f2bf(g);
    }
    *reinterpret_cast<u16x8*>(lrow + c * 8) = x;
  }
}

DLT_API int dlt_cross_entropy_fwd_bwd(bf16_t* logits, const int64_t* targets, const int64_t* n_valid,
                                      float* loss_rows, int M, int Vp, int V, hipStream_t st) {
  if (Vp % 8 || V > Vp) return -1;
  k_ce_fwd_bwd<<<M, 256, 0, st>>>(logits, targets, n_valid, loss_rows, M, Vp, V);
  DLT_CHECK_LAUNCH();
}
