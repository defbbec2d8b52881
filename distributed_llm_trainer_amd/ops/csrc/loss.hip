// Cross-entropy over the (padded) vocabulary with the gradient written in place.
//
// Reference: F.cross_entropy on shifted [B*(S-1), V] logits, fp32 under autocast
// (gpt.py:449-453; SURVEY §2.5 K11/K12: the fp32 log_softmax alone is 1.65 GB for
// small at B=8).  Here the bf16 logits buffer [M, Vp] from the lm_head GEMM is
// overwritten by
//   dlogits = (softmax(l) - onehot(target)) / n_valid       (0 for padded columns
// and for rows whose target is ignore_index), so no fp32 logits or separate
// softmax-backward kernel ever exist.
//
// k_ce_row: one block per row holds the whole row in registers, so HBM sees exactly
// one read and one write of the logits (the memory-bound minimum).  Default for
// Vp <= 57344: 1024 threads x 7 16-byte chunks, held to 64 VGPRs (8 waves per SIMD,
// two rows per CU in flight): 320 us vs 346 us per 8192 x 50304 call for 512 threads
// x 13 chunks (94 VGPRs, five waves per SIMD), bench step -0.1 to -0.2 ms
// (round-2 harness ab_ce.sh, in git history; DLT_CE_THREADS=512 selects the older shape).  Rows too long for
// registers fall back to k_ce_fwd_bwd (online max/sum pass + gradient pass).
#include "common.h"
#include <cstdlib>

template <int HK = 0>
__global__ __launch_bounds__(256) void k_ce_fwd_bwd(bf16_t* __restrict__ logits, const int64_t* __restrict__ targets,
                                                    const int64_t* __restrict__ n_valid, float* __restrict__ loss_rows,
                                                    int M, int Vp, int V, float gscale) {
  __shared__ float sm_m[4], sm_s[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  bf16_t* lrow = logits + (size_t)row * Vp;
  const int64_t tgt = targets[row];
  DLT_DASSERT(tgt == -100 || (tgt >= 0 && tgt < V));  // ignore_index or a real token
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
      v[e] = (c * 8 + e < V) ? h2f<HK>(x.v[e]) : -INFINITY;
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
  if (tid == 0) loss_rows[row] = valid ? (lse - h2f<HK>(lrow[tgt])) : 0.f;
  __syncthreads();  // everyone has read lrow[tgt] before it is overwritten
  const int64_t nv = *n_valid;
  const float inv_n = valid ? gscale / (float)(nv > 0 ? nv : 1) : 0.f;
  // pass 2: gradient in place
  for (int c = tid; c < nchunk; c += 256) {
    u16x8 x = *reinterpret_cast<const u16x8*>(lrow + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = c * 8 + e;
      float g = 0.f;
      if (col < V) {
        g = __expf(h2f<HK>(x.v[e]) - lse);
        if (col == tgt) g -= 1.f;
        g *= inv_n;
      }
      x.v[e] = f2h<HK>(g);
    }
    *reinterpret_cast<u16x8*>(lrow + c * 8) = x;
  }
}

// gscale: factor on the gradient only (1 for bf16; the fp16 path stores the gradient
// pre-multiplied by the loss scale so it does not underflow fp16, and the engine divides
// the scale back out where it applies dloss)
template <int CPT, int NTH = 512, bool CE_NT = false, int HK = 0>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(NTH == 1024 ? 8 : 1, 8))) void k_ce_row(bf16_t* __restrict__ logits, const int64_t* __restrict__ targets,
                                                const int64_t* __restrict__ n_valid, float* __restrict__ loss_rows,
                                                int M, int Vp, int V, float gscale) {
  // Per element only: max, one exp2 for the sum, one exp2 + scale for the gradient.
  // Column bounds are tested per 8-wide chunk (only the last chunk straddles V), and
  // the target column is patched by its owning thread per chunk, not per element.
  __shared__ float red[NTH / 64];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  bf16_t* lrow = logits + (size_t)row * Vp;
  const int64_t tgt = targets[row];
  DLT_DASSERT(tgt == -100 || (tgt >= 0 && tgt < V));  // ignore_index or a real token
  const bool valid = tgt >= 0 && tgt < V;
  const int tchunk = valid ? (int)(tgt >> 3) : -1;
  const int nchunk = Vp >> 3;
  const float L2E = 1.44269504088896340736f;
  uint4 x[CPT];  // 8 bf16 per chunk as 4 packed words
#pragma unroll
  for (int t = 0; t < CPT; ++t) {
    const int c = tid + NTH * t;
    if (c < nchunk) {
      if (CE_NT) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(lrow + c * 8);
        x[t] = make_uint4(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1),
                          __builtin_nontemporal_load(q + 2), __builtin_nontemporal_load(q + 3));
      } else {
        x[t] = *reinterpret_cast<const uint4*>(lrow + c * 8);
      }
    }
  }
  auto el = [&](int t, int e) -> float {
    const uint32_t w = e < 2 ? (e == 0 ? x[t].x : x[t].x) : e < 4 ? x[t].y : e < 6 ? x[t].z : x[t].w;
    if constexpr (HK == 0) return __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
    else return h2f<1>((uint16_t)((e & 1) ? (w >> 16) : (w & 0xffffu)));
  };
  // Keep only the raw bf16 words live across the passes (52 VGPRs at CPT 13): the
  // empty asm makes the compiler re-convert per pass instead of holding 104 floats.
  auto pin = [&]() {
#pragma unroll
    for (int t = 0; t < CPT; ++t) {
      asm volatile("" : "+v"(x[t].x), "+v"(x[t].y), "+v"(x[t].z), "+v"(x[t].w));
    }
  };
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < CPT; ++t) {
    const int c = tid + NTH * t;
    if (c * 8 + 8 <= V) {
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = fmaxf(mx, el(t, e));
    } else if (c < nchunk) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c * 8 + e < V) mx = fmaxf(mx, el(t, e));
    }
  }
  pin();
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  float gm = red[0];
#pragma unroll
  for (int w = 1; w < NTH / 64; ++w) gm = fmaxf(gm, red[w]);
  __syncthreads();
  const float nm2 = -gm * L2E;
  float sm = 0.f;
#pragma unroll
  for (int t = 0; t < CPT; ++t) {
    const int c = tid + NTH * t;
    if (c * 8 + 8 <= V) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sm += __builtin_amdgcn_exp2f(fmaf(el(t, e), L2E, nm2));
    } else if (c < nchunk) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c * 8 + e < V) sm += __builtin_amdgcn_exp2f(fmaf(el(t, e), L2E, nm2));
    }
  }
  pin();
  sm = wave_sum(sm);
  if (lane == 0) red[wid] = sm;
  __syncthreads();
  float gs = 0.f;
#pragma unroll
  for (int w = 0; w < NTH / 64; ++w) gs += red[w];
  const float lse = gm + __logf(gs);
  const int64_t nv = *n_valid;
  const float inv_n = valid ? gscale / (float)(nv > 0 ? nv : 1) : 0.f;
  const float nl2 = -lse * L2E;
#pragma unroll
  for (int t = 0; t < CPT; ++t) {
    const int c = tid + NTH * t;
    if (c < nchunk) {
      u16x8 o;
      if (c * 8 + 8 <= V) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o.v[e] = f2h<HK>(__builtin_amdgcn_exp2f(fmaf(el(t, e), L2E, nl2)) * inv_n);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          o.v[e] = f2h<HK>(c * 8 + e < V ? __builtin_amdgcn_exp2f(fmaf(el(t, e), L2E, nl2)) * inv_n : 0.f);
      }
      if (c == tchunk) {
        const int e = (int)(tgt & 7);
        float l = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) l = (j == e) ? el(t, j) : l;
        loss_rows[row] = lse - l;
        const uint16_t gt = f2h<HK>((__builtin_amdgcn_exp2f(fmaf(l, L2E, nl2)) - 1.f) * inv_n);
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = (j == e) ? gt : o.v[j];
      }
      if (CE_NT) {
        const uint4 w = __builtin_bit_cast(uint4, o);
        uint32_t* q = reinterpret_cast<uint32_t*>(lrow + c * 8);
        __builtin_nontemporal_store(w.x, q);
        __builtin_nontemporal_store(w.y, q + 1);
        __builtin_nontemporal_store(w.z, q + 2);
        __builtin_nontemporal_store(w.w, q + 3);
      } else {
        *reinterpret_cast<u16x8*>(lrow + c * 8) = o;
      }
    }
  }
  if (!valid && tid == 0) loss_rows[row] = 0.f;
}

template <int HK>
static void ce_launch(int wide, int nt, int cpt, hipStream_t st, bf16_t* logits, const int64_t* targets,
                      const int64_t* n_valid, float* loss_rows, int M, int Vp, int V, float gscale) {
#define CE_ARGS logits, targets, n_valid, loss_rows, M, Vp, V, gscale
  if (wide && (Vp / 8 + 1023) / 1024 <= 7) {  // 1024 threads x 7 chunks (Vp <= 57344)
    if (nt) k_ce_row<7, 1024, true, HK><<<M, 1024, 0, st>>>(CE_ARGS);
    else k_ce_row<7, 1024, false, HK><<<M, 1024, 0, st>>>(CE_ARGS);
    return;
  }
  if (cpt <= 1) k_ce_row<1, 512, false, HK><<<M, 512, 0, st>>>(CE_ARGS);
  else if (cpt <= 2) k_ce_row<2, 512, false, HK><<<M, 512, 0, st>>>(CE_ARGS);
  else if (cpt <= 4) k_ce_row<4, 512, false, HK><<<M, 512, 0, st>>>(CE_ARGS);
  else if (cpt <= 8) k_ce_row<8, 512, false, HK><<<M, 512, 0, st>>>(CE_ARGS);
  else if (cpt <= 13) k_ce_row<13, 512, false, HK><<<M, 512, 0, st>>>(CE_ARGS);
  else if (cpt <= 16) k_ce_row<16, 512, false, HK><<<M, 512, 0, st>>>(CE_ARGS);
  else k_ce_fwd_bwd<HK><<<M, 256, 0, st>>>(CE_ARGS);
#undef CE_ARGS
}

// hk: logits format (0 bf16, 1 fp16); gscale multiplies the in-place gradient
DLT_API int dlt_cross_entropy_fwd_bwd(bf16_t* logits, const int64_t* targets, const int64_t* n_valid,
                                      float* loss_rows, int M, int Vp, int V, float gscale, int hk, hipStream_t st) {
  if (Vp % 8 || V > Vp) return -1;
  const int cpt = (Vp / 8 + 511) / 512;
  static int wide = -1;
  if (wide < 0) {
    const char* e = getenv("DLT_CE_THREADS");
    wide = (e && atoi(e) == 512) ? 0 : 1;
  }
  // nontemporal logits loads / gradient stores (the [M, Vp] buffer is far larger than
  // the Infinity Cache): 305 vs 319 us per 8192-row call, step -0.06 / -0.14 ms in two
  // same-box pairs; DLT_CE_NT=0 selects plain accesses
  static int nt = -1;
  if (nt < 0) {
    const char* e = getenv("DLT_CE_NT");
    nt = (e && atoi(e) == 0) ? 0 : 1;
  }
  DLT_HK_DISPATCH(hk, ce_launch<HKC>(wide, nt, cpt, st, logits, targets, n_valid, loss_rows, M, Vp, V, gscale));
  DLT_CHECK_LAUNCH();
}
