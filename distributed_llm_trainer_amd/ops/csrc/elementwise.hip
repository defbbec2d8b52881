// Memory-bound fused elementwise kernels: embedding gather / scatter-add,
// RoPE + QKV head split (fwd/bwd), SwiGLU (fwd/bwd).  All move 8-16 B per lane.
//
// Reference ops replaced: K1 embedding (gpt.py:438), K4 RoPE
// (gpt.py:144-147,195-196) together with the view/transpose of gpt.py:190-192,
// K8 silu*mul (gpt.py:280).
#include "common.h"

// ---------------------------------------------------------------- embedding
// out[m, :] = float(W[ids[m], :]); W is fp32 (wdt=0), bf16 (wdt=1) or fp16 (wdt=2).
__global__ __launch_bounds__(256) void k_embedding_fwd(const int64_t* __restrict__ ids, const void* __restrict__ W,
                                                       int wdt, float* __restrict__ out, int M, int H, int V) {
  const int q = H >> 2;  // float4 per row
  const size_t total = (size_t)M * q;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / q);
    const int c = (int)(i % q);
    const int64_t id = ids[m];
    DLT_DASSERT(id >= 0 && id < V);
    float4 v;
    if (wdt == 0) {
      v = *(reinterpret_cast<const float4*>(W) + (size_t)id * q + c);
    } else if (wdt == 1) {
      const u16x4 b = *(reinterpret_cast<const u16x4*>(W) + (size_t)id * q + c);
      v = make_float4(bf2f(b.v[0]), bf2f(b.v[1]), bf2f(b.v[2]), bf2f(b.v[3]));
    } else {
      const u16x4 b = *(reinterpret_cast<const u16x4*>(W) + (size_t)id * q + c);
      v = make_float4(h2f<1>(b.v[0]), h2f<1>(b.v[1]), h2f<1>(b.v[2]), h2f<1>(b.v[3]));
    }
    *(reinterpret_cast<float4*>(out) + i) = v;
  }
}

// Deterministic scatter-add dW[v, :] += sum of dout[m, :] over ids[m] == v (SURVEY K1:
// sorted segment-sum, no float atomics, so gradients are bitwise reproducible).  The
// ids arrive stably sorted (sids, with perm = original positions), so the rows of one
// token id form a run in increasing m.  Pass 1: one wave per chunk of EMB_CH sorted
// positions walks the runs of its chunk; a run inside the chunk is added to dW directly
// (its only writer), a run cut by a chunk edge leaves a partial in ws[chunk][0] (cut on
// the left) or ws[chunk][1] (cut on the right only).  Pass 2: the chunk where a cut run
// starts adds its partial and the following chunks' left partials, in chunk order.
// Lane = 4 columns per 256-column slice; the run walk is wave-uniform.
#define EMB_CH 4
__global__ __launch_bounds__(256) void k_embedding_bwd_runs(const int* __restrict__ sids,
                                                            const int64_t* __restrict__ perm,
                                                            const float* __restrict__ dout, float* __restrict__ dW,
                                                            float* __restrict__ ws, int M, int H, int V) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int p0 = c * EMB_CH;
  if (p0 >= M) return;
  const int p1 = min(M, p0 + EMB_CH);
  int s = p0;
  while (s < p1) {
    const int v = sids[s];
    DLT_DASSERT(v >= 0 && v < V);
    int e = s + 1;
    while (e < p1 && sids[e] == v) ++e;
    const bool cut_l = s == p0 && p0 > 0 && sids[p0 - 1] == v;
    const bool cut_r = e == p1 && p1 < M && sids[p1] == v;
    float* dst = cut_l ? ws + (size_t)(2 * c) * H : cut_r ? ws + (size_t)(2 * c + 1) * H : dW + (size_t)v * H;
    for (int col = lane * 4; col < H; col += 256) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int q = s; q < e; ++q) {
        const float4 d = *reinterpret_cast<const float4*>(dout + (size_t)perm[q] * H + col);
        a.x += d.x; a.y += d.y; a.z += d.z; a.w += d.w;
      }
      float4* o = reinterpret_cast<float4*>(dst + col);
      if (!(cut_l || cut_r)) {
        const float4 w = *o;
        a.x += w.x; a.y += w.y; a.z += w.z; a.w += w.w;
      }
      *o = a;
    }
    s = e;
  }
}

__global__ __launch_bounds__(256) void k_embedding_bwd_spans(const int* __restrict__ sids,
                                                             const float* __restrict__ ws, float* __restrict__ dW,
                                                             int M, int H) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int p0 = c * EMB_CH;
  if (p0 >= M) return;
  const int p1 = p0 + EMB_CH;
  if (p1 >= M) return;
  const int v = sids[p1 - 1];
  if (sids[p1] != v) return;                               // last run not cut on the right
  if (sids[p0] == v && p0 > 0 && sids[p0 - 1] == v) return;  // run started in an earlier chunk
  int c_end = c + 1;                                         // chunks [c+1, c_end] hold the rest
  while ((c_end + 1) * EMB_CH < M && sids[(c_end + 1) * EMB_CH] == v) ++c_end;
  for (int col = lane * 4; col < H; col += 256) {
    float4 a = *reinterpret_cast<const float4*>(ws + (size_t)(2 * c + 1) * H + col);
    int k = c + 1;
    for (; k + 7 <= c_end; k += 8) {  // 8 independent loads in flight, added in chunk order
      float4 d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) d[u] = *reinterpret_cast<const float4*>(ws + (size_t)(2 * (k + u)) * H + col);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a.x += d[u].x; a.y += d[u].y; a.z += d[u].z; a.w += d[u].w;
      }
    }
    for (; k <= c_end; ++k) {
      const float4 d = *reinterpret_cast<const float4*>(ws + (size_t)(2 * k) * H + col);
      a.x += d.x; a.y += d.y; a.z += d.z; a.w += d.w;
    }
    float4* o = reinterpret_cast<float4*>(dW + (size_t)v * H + col);
    const float4 w = *o;
    a.x += w.x; a.y += w.y; a.z += w.z; a.w += w.w;
    *o = a;
  }
}

DLT_API int dlt_embedding_fwd(const int64_t* ids, const void* W, int wdt, float* out, int M, int H, int V,
                              hipStream_t s) {
  if (H % 4) return -1;
  const size_t total = (size_t)M * (H / 4);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  k_embedding_fwd<<<blocks, 256, 0, s>>>(ids, W, wdt, out, M, H, V);
  DLT_CHECK_LAUNCH();
}

// sids/perm: torch.sort(int32 ids, stable=True); ws: 2 * ceil(M / EMB_CH) * H floats.
DLT_API int dlt_embedding_bwd(const int* sids, const int64_t* perm, const float* dout, float* dW, float* ws,
                              int M, int H, int V, hipStream_t s) {
  if (H % 4 || M <= 0) return -1;
  const int chunks = (M + EMB_CH - 1) / EMB_CH;
  const int blocks = (chunks + 3) / 4;
  k_embedding_bwd_runs<<<blocks, 256, 0, s>>>(sids, perm, dout, dW, ws, M, H, V);
  k_embedding_bwd_spans<<<blocks, 256, 0, s>>>(sids, ws, dW, M, H);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_embedding_bwd_chunk() { return EMB_CH; }

// ---------------------------------------------------------------- RoPE
// qkv [B*S, 3, nh, hd] (bf16) -> q, k, v [B, nh, S, hd]; q, k rotated (NeoX half split)
// in fp32 with cos/sin tables [S, hd/2].  One thread = 4 rotary pairs of one head.
// One thread = one 8-wide chunk of each rotation half (16-B vectors; the partner
// element of column j is j + hd/2 in NeoX rotate_half).  32-bit index math only
// (64-bit div/mod is emulated on the GPU and cost ~30 % of this kernel).
template <int HK = 0>
__global__ __launch_bounds__(256) void k_rope_qkv_fwd(const bf16_t* __restrict__ qkv, const float* __restrict__ cosT,
                                                      const float* __restrict__ sinT, bf16_t* __restrict__ q,
                                                      bf16_t* __restrict__ k, bf16_t* __restrict__ v,
                                                      int B, int S, int nh, int hd) {
  const int half = hd >> 1;
  const int cpr = half >> 3;  // 8-wide chunks per rotation half
  const int total = B * S * 3 * nh * cpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = (i % cpr) * 8;
    int r = i / cpr;
    const int h = r % nh;
    r /= nh;
    const int sec = r % 3;
    const int m = r / 3;
    const int s = m % S, b = m / S;
    const bf16_t* src = qkv + (size_t)m * (3 * nh * hd) + (sec * nh + h) * hd;
    const u16x8 a = *reinterpret_cast<const u16x8*>(src + j);
    const u16x8 c = *reinterpret_cast<const u16x8*>(src + half + j);
    bf16_t* dst = (sec == 0 ? q : (sec == 1 ? k : v)) + ((size_t)(b * nh + h) * S + s) * hd;
    u16x8 o1 = a, o2 = c;
    if (sec != 2) {
      const float* cp = cosT + s * half + j;
      const float* sp = sinT + s * half + j;
      const float4 c0 = *reinterpret_cast<const float4*>(cp), c1 = *reinterpret_cast<const float4*>(cp + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(sp), s1 = *reinterpret_cast<const float4*>(sp + 4);
      const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x1 = h2f<HK>(a.v[e]), x2 = h2f<HK>(c.v[e]);
        o1.v[e] = f2h<HK>(x1 * cc[e] - x2 * ss[e]);
        o2.v[e] = f2h<HK>(x2 * cc[e] + x1 * ss[e]);
      }
    }
    *reinterpret_cast<u16x8*>(dst + j) = o1;
    *reinterpret_cast<u16x8*>(dst + half + j) = o2;
  }
}

// dq, dk, dv [B, nh, S, hd] -> dqkv [B*S, 3*nh*hd] (inverse rotation for dq, dk).
// dq may be fp32 (dqf != nullptr) or bf16.
template <int HK = 0>
__global__ __launch_bounds__(256) void k_rope_qkv_bwd(const bf16_t* __restrict__ dq, const float* __restrict__ dqf,
                                                      const bf16_t* __restrict__ dk, const bf16_t* __restrict__ dv,
                                                      const float* __restrict__ cosT, const float* __restrict__ sinT,
                                                      bf16_t* __restrict__ dqkv, int B, int S, int nh, int hd) {
  const int half = hd >> 1;
  const int cpr = half >> 3;
  const int total = B * S * 3 * nh * cpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = (i % cpr) * 8;
    int r = i / cpr;
    const int h = r % nh;
    r /= nh;
    const int sec = r % 3;
    const int m = r / 3;
    const int s = m % S, b = m / S;
    const size_t soff = ((size_t)(b * nh + h) * S + s) * hd;
    float g1[8], g2[8];
    if (sec == 0 && dqf) {
      const float* p = dqf + soff;
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const float4 a = *reinterpret_cast<const float4*>(p + j + e);
        const float4 c = *reinterpret_cast<const float4*>(p + half + j + e);
        g1[e] = a.x; g1[e + 1] = a.y; g1[e + 2] = a.z; g1[e + 3] = a.w;
        g2[e] = c.x; g2[e + 1] = c.y; g2[e + 2] = c.z; g2[e + 3] = c.w;
      }
    } else {
      const bf16_t* src = (sec == 0 ? dq : (sec == 1 ? dk : dv)) + soff;
      const u16x8 a = *reinterpret_cast<const u16x8*>(src + j);
      const u16x8 c = *reinterpret_cast<const u16x8*>(src + half + j);
#pragma unroll
      for (int e = 0; e < 8; ++e) { g1[e] = h2f<HK>(a.v[e]); g2[e] = h2f<HK>(c.v[e]); }
    }
    u16x8 o1, o2;
    if (sec == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { o1.v[e] = f2h<HK>(g1[e]); o2.v[e] = f2h<HK>(g2[e]); }
    } else {
      const float* cp = cosT + s * half + j;
      const float* sp = sinT + s * half + j;
      const float4 c0 = *reinterpret_cast<const float4*>(cp), c1 = *reinterpret_cast<const float4*>(cp + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(sp), s1 = *reinterpret_cast<const float4*>(sp + 4);
      const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o1.v[e] = f2h<HK>(g1[e] * cc[e] + g2[e] * ss[e]);
        o2.v[e] = f2h<HK>(g2[e] * cc[e] - g1[e] * ss[e]);
      }
    }
    bf16_t* dst = dqkv + (size_t)m * (3 * nh * hd) + (sec * nh + h) * hd;
    *reinterpret_cast<u16x8*>(dst + j) = o1;
    *reinterpret_cast<u16x8*>(dst + half + j) = o2;
  }
}

// In-place RoPE of the packed [B*S, 3, nh, hd] QKV GEMM output: the q and k column
// blocks (2*nh contiguous heads per row) are rotated, v is untouched.  The attention
// kernels then read q/k/v straight from this buffer (dlt_attn_fwd_ex), so no head-major
// copies are written (2/3 of the traffic of k_rope_qkv_fwd, and its backward
// disappears into the attention epilogue).
template <int HK = 0>
__global__ __launch_bounds__(256) void k_rope_qk_inplace(bf16_t* __restrict__ qkv, const float* __restrict__ cosT,
                                                         const float* __restrict__ sinT, int M, int S, int nh,
                                                         int hd) {
  const int half = hd >> 1;
  const int cpr = half >> 3;  // 8-wide chunks per rotation half
  const int hq = 2 * nh;      // rotated heads per row (q then k)
  const int total = M * hq * cpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = (i % cpr) * 8;
    const int r = i / cpr;
    const int hh = r % hq;
    const int m = r / hq;
    const int s = m % S;
    bf16_t* p = qkv + (size_t)m * (3 * nh * hd) + hh * hd;
    const u16x8 a = *reinterpret_cast<const u16x8*>(p + j);
    const u16x8 c = *reinterpret_cast<const u16x8*>(p + half + j);
    const float* cp = cosT + s * half + j;
    const float* sp = sinT + s * half + j;
    const float4 c0 = *reinterpret_cast<const float4*>(cp), c1 = *reinterpret_cast<const float4*>(cp + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(sp), s1 = *reinterpret_cast<const float4*>(sp + 4);
    const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    u16x8 o1, o2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x1 = h2f<HK>(a.v[e]), x2 = h2f<HK>(c.v[e]);
      o1.v[e] = f2h<HK>(x1 * cc[e] - x2 * ss[e]);
      o2.v[e] = f2h<HK>(x2 * cc[e] + x1 * ss[e]);
    }
    *reinterpret_cast<u16x8*>(p + j) = o1;
    *reinterpret_cast<u16x8*>(p + half + j) = o2;
  }
}

static inline int ew_blocks(size_t total) {
  size_t b = (total + 255) / 256;
  return (int)(b > 16384 ? 16384 : (b == 0 ? 1 : b));
}

DLT_API int dlt_rope_qkv_fwd(const bf16_t* qkv, const float* cosT, const float* sinT, bf16_t* q, bf16_t* k,
                             bf16_t* v, int B, int S, int nh, int hd, int hk, hipStream_t st) {
  if (hd % 16 || (long)B * S * 3 * nh * hd >= (1L << 31)) return -1;
  const size_t total = (size_t)B * S * 3 * nh * (hd / 16);
  DLT_HK_DISPATCH(hk, k_rope_qkv_fwd<HKC><<<ew_blocks(total), 256, 0, st>>>(qkv, cosT, sinT, q, k, v, B, S, nh, hd));
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_rope_qk_inplace(bf16_t* qkv, const float* cosT, const float* sinT, int M, int S, int nh, int hd,
                                int hk, hipStream_t st) {
  if (hd % 16 || S <= 0 || M % S || (long)M * 3 * nh * hd >= (1L << 31)) return -1;
  const size_t total = (size_t)M * 2 * nh * (hd / 16);
  DLT_HK_DISPATCH(hk, k_rope_qk_inplace<HKC><<<ew_blocks(total), 256, 0, st>>>(qkv, cosT, sinT, M, S, nh, hd));
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_rope_qkv_bwd(const bf16_t* dq, const float* dqf, const bf16_t* dk, const bf16_t* dv,
                             const float* cosT, const float* sinT, bf16_t* dqkv, int B, int S, int nh, int hd, int hk,
                             hipStream_t st) {
  if (hd % 16 || (long)B * S * 3 * nh * hd >= (1L << 31)) return -1;
  const size_t total = (size_t)B * S * 3 * nh * (hd / 16);
  DLT_HK_DISPATCH(hk, k_rope_qkv_bwd<HKC><<<ew_blocks(total), 256, 0, st>>>(dq, dqf, dk, dv, cosT, sinT, dqkv, B, S,
                                                                             nh, hd));
  DLT_CHECK_LAUNCH();
}

// ---------------------------------------------------------------- SwiGLU
__device__ __forceinline__ float sigmoidf_(float x) { return dlt_sigmoid(x); }

// gu [M, 2I] = [gate | up] -> a [M, I] = silu(gate) * up
template <int HK = 0>
__global__ __launch_bounds__(256) void k_swiglu_fwd(const bf16_t* __restrict__ gu, bf16_t* __restrict__ a, int M, int I) {
  const int q = I >> 3;
  const size_t total = (size_t)M * q;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / q;
    const int c = (int)(i % q) * 8;
    const u16x8 g = *reinterpret_cast<const u16x8*>(gu + m * 2 * I + c);
    const u16x8 u = *reinterpret_cast<const u16x8*>(gu + m * 2 * I + I + c);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gv = h2f<HK>(g.v[e]);
      o.v[e] = f2h<HK>(gv * sigmoidf_(gv) * h2f<HK>(u.v[e]));
    }
    *reinterpret_cast<u16x8*>(a + m * I + c) = o;
  }
}

// s_out (optional): also writes s = silu(g) * u with the forward's exact arithmetic
// (k_swiglu_fwd, same bits) -- the engine's ffbb window keeps s only in a short slot ring
// filled here instead of one [M, I] slot per layer from the forward.
template <int HK = 0>
__global__ __launch_bounds__(256) void k_swiglu_bwd(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ da,
                                                    bf16_t* __restrict__ dgu, bf16_t* __restrict__ s_out, int M,
                                                    int I) {
  const int q = I >> 3;
  const size_t total = (size_t)M * q;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / q;
    const int c = (int)(i % q) * 8;
    const u16x8 g = *reinterpret_cast<const u16x8*>(gu + m * 2 * I + c);
    const u16x8 u = *reinterpret_cast<const u16x8*>(gu + m * 2 * I + I + c);
    const u16x8 d = *reinterpret_cast<const u16x8*>(da + m * I + c);
    u16x8 og, ou, os;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gv = h2f<HK>(g.v[e]), uv = h2f<HK>(u.v[e]), dv = h2f<HK>(d.v[e]);
      const float sg = sigmoidf_(gv);
      og.v[e] = f2h<HK>(dv * uv * sg * (1.f + gv * (1.f - sg)));
      ou.v[e] = f2h<HK>(dv * gv * sg);
      os.v[e] = f2h<HK>(gv * sg * uv);
    }
    *reinterpret_cast<u16x8*>(dgu + m * 2 * I + c) = og;
    *reinterpret_cast<u16x8*>(dgu + m * 2 * I + I + c) = ou;
    if (s_out) *reinterpret_cast<u16x8*>(s_out + m * I + c) = os;
  }
}

// y = x * (*scale) for a bf16 tensor and a device fp32 scalar (the autograd output
// gradient), one pass -- replaces an upcast + multiply + downcast kernel chain.
template <int HK = 0>
__global__ __launch_bounds__(256) void k_scale_bf16(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                    long n8, const float* __restrict__ scale, float mul) {
  const float sc = *scale * mul;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    u16x8 v = reinterpret_cast<const u16x8*>(x)[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) v.v[e] = f2h<HK>(h2f<HK>(v.v[e]) * sc);
    reinterpret_cast<u16x8*>(y)[i] = v;
  }
}

DLT_API int dlt_scale_bf16(const bf16_t* x, bf16_t* y, long n, const float* scale, float mul, int hk,
                           hipStream_t st) {
  if (n % 8) return -1;
  const long n8 = n / 8;
  const int blocks = (int)((n8 + 255) / 256 < 4096 ? (n8 + 255) / 256 : 4096);
  DLT_HK_DISPATCH(hk, k_scale_bf16<HKC><<<blocks, 256, 0, st>>>(x, y, n8, scale, mul));
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_swiglu_fwd(const bf16_t* gu, bf16_t* a, int M, int I, int hk, hipStream_t st) {
  if (I % 8) return -1;
  DLT_HK_DISPATCH(hk, k_swiglu_fwd<HKC><<<ew_blocks((size_t)M * (I / 8)), 256, 0, st>>>(gu, a, M, I));
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_swiglu_bwd(const bf16_t* gu, const bf16_t* da, bf16_t* dgu, bf16_t* s_out, int M, int I, int hk,
                           hipStream_t st) {
  if (I % 8) return -1;
  DLT_HK_DISPATCH(hk, k_swiglu_bwd<HKC><<<ew_blocks((size_t)M * (I / 8)), 256, 0, st>>>(gu, da, dgu, s_out, M, I));
  DLT_CHECK_LAUNCH();
}

// ---------------------------------------------------------------- split-K sum
// dw[i] += sum_{s < splits} part[s * n + i], summed in fixed order (deterministic, no
// atomics: DDP replicas must stay bit-identical).  float4 per lane; part comes from the
// strided-batched split-K weight-gradient GEMM (ops/gemm.py wgrad_acc).  n % 4 == 0.
__global__ __launch_bounds__(256) void k_splitk_acc(const float4* __restrict__ part, float4* __restrict__ dw,
                                                    long n4, int splits) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 a = dw[i];
    for (int s = 0; s < splits; ++s) {
      const float4 p = part[(long)s * n4 + i];
      a.x += p.x;
      a.y += p.y;
      a.z += p.z;
      a.w += p.w;
    }
    dw[i] = a;
  }
}

// out[i] = bf16(sum_{s < splits} part[s * n + i]) -- the split-K weight gradient written
// straight in the reduce dtype (FSDP: the per-micro-step unit gradient IS the
// reduce-scatter send buffer, no fp32 zero / accumulate / cast passes).  Fixed order.
template <int HK = 0>
__global__ __launch_bounds__(256) void k_splitk_sum_bf16(const float4* __restrict__ part, uint2* __restrict__ out,
                                                         long n4, int splits) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 a = part[i];
    for (int s = 1; s < splits; ++s) {
      const float4 p = part[(long)s * n4 + i];
      a.x += p.x;
      a.y += p.y;
      a.z += p.z;
      a.w += p.w;
    }
    out[i] = uint2{(uint32_t)f2h<HK>(a.x) | ((uint32_t)f2h<HK>(a.y) << 16),
                   (uint32_t)f2h<HK>(a.z) | ((uint32_t)f2h<HK>(a.w) << 16)};
  }
}

// hk: output format (0 bf16, 1 fp16)
DLT_API int dlt_splitk_sum_bf16(const float* part, bf16_t* out, long n, int splits, int hk, hipStream_t s) {
  if (n <= 0 || (n & 3) || splits < 1) return -1;
  const long n4 = n / 4;
  const int blocks = (int)std::min<long>((n4 + 255) / 256, 2048);
  DLT_HK_DISPATCH(hk, k_splitk_sum_bf16<HKC><<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(part),
                                                                   reinterpret_cast<uint2*>(out), n4, splits));
  return (int)hipGetLastError();
}

DLT_API int dlt_splitk_acc(const float* part, float* dw, long n, int splits, hipStream_t s) {
  if (n <= 0 || (n & 3) || splits < 1) return -1;
  const long n4 = n / 4;
  const int blocks = (int)std::min<long>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(k_splitk_acc, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const float4*>(part),
                     reinterpret_cast<float4*>(dw), n4, splits);
  return (int)hipGetLastError();
}
