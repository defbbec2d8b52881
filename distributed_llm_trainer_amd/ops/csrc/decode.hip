// Fused one-token decode step (KV-cached generation, eval/decode.py) for gfx950.
//
// The reference's GPT.generate (gpt.py:457-484) re-runs the whole forward for every new
// token.  The KV-cached decoder needs, per layer and token, five
// GEMV-sized steps; written as ATen ops they were ~25 small kernels per layer (~200 per
// token, launch/latency bound even inside a HIP graph: 1.8 ms per token for GPT-2 small).
// Here each step is ONE kernel (5 per layer + the head), all of them bandwidth-shaped:
//
//   dec_norm_qkv    : h -> RMSNorm -> QKV GEMV -> RoPE(q, k) -> K/V cache row at `pos`, q
//   dec_attn        : q . K[0..pos]^T -> softmax -> . V      (one workgroup per (b, head))
//   dec_gemv_res    : h += o . Wo^T  /  h += s . Wdown^T      (residual add in fp32)
//   dec_norm_gu     : h -> RMSNorm -> gate/up GEMV -> SwiGLU -> s
//   dec_norm_head   : h -> RMSNorm -> lm_head GEMV -> fp32 logits
//
// GEMV shape: a wave computes 4 output rows at once, lanes across K (16-byte weight loads:
// the weight stream, which dominates the bytes, is coalesced, and all 4 rows' loads are in
// flight before any reduction), 16 rows per workgroup so even the 768-row projections
// spread over 48+ workgroups; the B <= 8 activation rows are staged once per workgroup in
// LDS as bf16; fp32 accumulation and a 6-step xor-shuffle reduction.  Numerics follow the eager decode path (eval/decode.py forward_cached): the
// normed activations and every GEMV output are rounded to bf16 like torch's bf16 matmul,
// the residual stream and softmax are fp32.  `pos` is a device scalar so the step can be
// captured once in a HIP graph and replayed per token.
#include "common.h"

namespace {

constexpr int DEC_NT = 256;  // 4 waves

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float bf_round(float x) { return bf2f(f2bf(x)); }

__device__ __forceinline__ float norm_w(const void* w, int wbf16, int i) {
  return wbf16 ? bf2f(reinterpret_cast<const bf16_t*>(w)[i]) : reinterpret_cast<const float*>(w)[i];
}

// xs[b][k] (bf16, LDS) = bf16(h[b][k] * rsqrt(mean(h[b]^2) + eps) * w[k]) for b < B.
// float4 loads, every row's loads issued before the reductions (the per-element loop
// was a chain of dependent round trips: most of a kernel's time).
template <int B>
__device__ void stage_normed(const float* __restrict__ h, int K, const void* w, int wbf16, float eps, bf16_t* xs,
                             float* red) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nch = K >> 2;  // float4 chunks per row (K % 8 == 0)
  float ss[B];
#pragma unroll
  for (int b = 0; b < B; ++b) {
    ss[b] = 0.f;
#pragma unroll 2
    for (int c = tid; c < nch; c += DEC_NT) {
      const float4 x = *reinterpret_cast<const float4*>(h + (size_t)b * K + 4 * c);
      ss[b] += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    }
  }
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const float t = wave_sum64(ss[b]);
    if (lane == 0) red[b * 4 + wid] = t;
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const float rstd = rsqrtf((red[b * 4] + red[b * 4 + 1] + red[b * 4 + 2] + red[b * 4 + 3]) / (float)K + eps);
#pragma unroll 2
    for (int c = tid; c < nch; c += DEC_NT) {
      const float4 x = *reinterpret_cast<const float4*>(h + (size_t)b * K + 4 * c);
      u16x4 y;
      y.v[0] = f2bf(x.x * rstd * norm_w(w, wbf16, 4 * c));
      y.v[1] = f2bf(x.y * rstd * norm_w(w, wbf16, 4 * c + 1));
      y.v[2] = f2bf(x.z * rstd * norm_w(w, wbf16, 4 * c + 2));
      y.v[3] = f2bf(x.w * rstd * norm_w(w, wbf16, 4 * c + 3));
      *reinterpret_cast<u16x4*>(xs + b * K + 4 * c) = y;
    }
  }
  __syncthreads();
}

// xs[b][k] = x[b][k] (bf16 global -> LDS), 16-byte chunks, unrolled so the loads overlap
template <int B>
__device__ void stage_copy(const bf16_t* __restrict__ x, int K, bf16_t* xs) {
  const int n = B * K / 8;
#pragma unroll 4
  for (int c = threadIdx.x; c < n; c += DEC_NT)
    *reinterpret_cast<u16x8*>(xs + 8 * c) = *reinterpret_cast<const u16x8*>(x + 8 * c);
  __syncthreads();
}

// Weight-stream load: each weight byte is read by one workgroup once per token, so the
// loads are nontemporal (no point keeping the lines in L2 for a reuse that never comes).
__device__ __forceinline__ u16x8 ld_w8(const bf16_t* p) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  u16x8 r;
  __builtin_memcpy(&r, &t, 16);
  return r;
}

// acc[r][b] = sum_k W_r[k] * xs[b][k] for NR rows at once, the whole wave (lanes across K):
// every row's weight loads are issued before any reduction, so a wave has NR x K/512
// 16-byte loads in flight (one load round trip per group instead of one per row).  The
// first PRE 512-element slices of every row are loaded by rows_pre() BEFORE the workgroup
// stages its activations, so the weight stream's HBM latency overlaps the staging.
template <int NR, int PRE>
struct RowsPre {
  u16x8 wv[NR][PRE];
};

template <int NR, int PRE>
__device__ __forceinline__ void rows_pre(const bf16_t* const (&wrow)[NR], int K, RowsPre<NR, PRE>& pre) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < PRE; ++i) {
    const int c = i * 64 + lane;
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (c * 8 < K) pre.wv[r][i] = ld_w8(wrow[r] + c * 8);
  }
}

template <int B, int NR>
__device__ __forceinline__ void fma_slice(const u16x8 (&wv)[NR], const bf16_t* xs, int K, int c, float (&acc)[NR][B]) {
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const u16x8 xv = *reinterpret_cast<const u16x8*>(xs + b * K + c * 8);
    float xf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xf[e] = bf2f(xv.v[e]);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[r][b] = fmaf(bf2f(wv[r].v[e]), xf[e], acc[r][b]);
  }
}

template <int B, int NR, int PRE>
__device__ __forceinline__ void rows_dot(const bf16_t* const (&wrow)[NR], int K, const bf16_t* xs,
                                         const RowsPre<NR, PRE>& pre, float (&acc)[NR][B]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.f;
#pragma unroll
  for (int i = 0; i < PRE; ++i) {
    const int c = i * 64 + lane;
    if (c * 8 < K) {
      u16x8 wv[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) wv[r] = pre.wv[r][i];
      fma_slice<B, NR>(wv, xs, K, c, acc);
    }
  }
#pragma unroll 4
  for (int c0 = PRE * 64; c0 * 8 < K; c0 += 64) {
    const int c = c0 + lane;
    if (c * 8 < K) {
      u16x8 wv[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) wv[r] = ld_w8(wrow[r] + c * 8);
      fma_slice<B, NR>(wv, xs, K, c, acc);
    }
  }
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = wave_sum64(acc[r][b]);
}

}  // namespace

// grid (3 * nh * 4): workgroup g owns dims {8c..8c+7} u {8c+32..8c+39} (c = g % 4: the 8
// NeoX RoPE pairs of a quarter head) of head (g / 4) % nh of block g / (4 nh) (0 q, 1 k,
// 2 v) -- 16 rows, 4 per wave, one load round trip.
template <int B>
__global__ __launch_bounds__(DEC_NT) void k_dec_norm_qkv(const float* __restrict__ h, const void* __restrict__ lnw,
                                                         int wbf16, float eps, const bf16_t* __restrict__ wqkv,
                                                         const float* __restrict__ cosT, const float* __restrict__ sinT,
                                                         const long* __restrict__ posp, bf16_t* __restrict__ qout,
                                                         bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int H, int nh,
                                                         int maxS) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(dsm);                       // [B][H]
  float* red = reinterpret_cast<float*>(dsm + (size_t)B * H * 2);     // [B][4]
  float* outv = red + B * 4;                                          // [B][16]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int quarter = blockIdx.x & 3, hb = blockIdx.x >> 2;
  const int blk = hb / nh, head = hb % nh;
  // local row l (0..15) -> head dim: l < 8 ? 8 quarter + l : 32 + 8 quarter + (l - 8)
  auto dim_of = [&](int l) { return (l < 8 ? 0 : 32) + 8 * quarter + (l & 7); };
  const bf16_t* rows[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rows[r] = wqkv + (size_t)(blk * H + head * 64 + dim_of(wid * 4 + r)) * H;
  RowsPre<4, 2> pre;
  rows_pre<4, 2>(rows, H, pre);
  stage_normed<B>(h, H, lnw, wbf16, eps, xs, red);
  float acc[4][B];
  rows_dot<B, 4, 2>(rows, H, xs, pre, acc);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int b = 0; b < B; ++b) outv[b * 16 + wid * 4 + r] = bf_round(acc[r][b]);  // torch bf16 matmul output
  }
  __syncthreads();
  const int pos = (int)posp[0];
  // the cache row and the RoPE table row must exist (a caller bug otherwise: the host
  // keeps pos < max_seq_len, see eval/decode.py); never write past the cache
  DLT_DASSERT(pos >= 0 && pos < maxS);
  if (pos < 0 || pos >= maxS) return;
  if (threadIdx.x < B * 16) {
    const int b = threadIdx.x >> 4, l = threadIdx.x & 15, d = dim_of(l);
    float y = outv[b * 16 + l];
    if (blk < 2) {  // NeoX RoPE on q and k: the partner of dim d is d +- 32 = local row l +- 8
      const int j = d & 31;
      const float c = cosT[(size_t)pos * 32 + j], sn = sinT[(size_t)pos * 32 + j];
      const float x1 = outv[b * 16 + (l & 7)], x2 = outv[b * 16 + 8 + (l & 7)];
      y = l < 8 ? x1 * c - x2 * sn : x2 * c + x1 * sn;
    }
    if (blk == 0)
      qout[(size_t)b * H + head * 64 + d] = f2bf(y);
    else
      (blk == 1 ? kc : vc)[(((size_t)b * nh + head) * maxS + pos) * 64 + d] = f2bf(y);
  }
}

// grid (B * nh): one (b, head).  q [B, H] bf16 (head-major 64-blocks), caches [B, nh, maxS, 64].
// Scores in fp32 (lane = key), softmax over keys 0..pos, then o (lane = dim) summed across
// the 4 waves in LDS.
__global__ __launch_bounds__(DEC_NT) void k_dec_attn(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                     const bf16_t* __restrict__ vc, const long* __restrict__ posp,
                                                     bf16_t* __restrict__ o, int H, int nh, int maxS, float scale) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  float* sc = reinterpret_cast<float*>(dsm);       // [maxS] scores -> probabilities
  float* red = sc + maxS;                          // [8]
  float* oacc = red + 8;                           // [4][64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x / nh, head = blockIdx.x % nh;
  DLT_DASSERT(posp[0] >= 0 && posp[0] < maxS);
  const int len = (int)(posp[0] < maxS ? posp[0] + 1 : maxS);  // sc[] holds maxS scores
  const bf16_t* K = kc + ((size_t)b * nh + head) * maxS * 64;
  const bf16_t* V = vc + ((size_t)b * nh + head) * maxS * 64;
  float qv[64];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const u16x8 t = *reinterpret_cast<const u16x8*>(q + (size_t)b * H + head * 64 + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[c * 8 + e] = bf2f(t.v[e]);
  }
  float mx = -INFINITY;
  for (int j = tid; j < len; j += DEC_NT) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const u16x8 t = *reinterpret_cast<const u16x8*>(K + (size_t)j * 64 + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s = fmaf(qv[c * 8 + e], bf2f(t.v[e]), s);
    }
    s *= scale;
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
#pragma unroll
  for (int o2 = 32; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int j = tid; j < len; j += DEC_NT) {
    const float p = __expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = wave_sum64(sum);
  __syncthreads();  // every red[] max read before it is overwritten
  if (lane == 0) red[4 + wid] = sum;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  // o[d] = sum_j p_j v_j[d]: lane (js, dc) = (tid / 8, tid % 8) loads dims 8dc..8dc+7 of
  // keys j = js, js + 32, ... (16-byte loads, all in flight), then the 32 key slots are
  // summed: 3 xor-shuffle steps inside the wave, the 4 waves through LDS.
  const int dc = tid & 7, js = tid >> 3;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int j = js; j < len; j += DEC_NT / 8) {
    const u16x8 t = *reinterpret_cast<const u16x8*>(V + (size_t)j * 64 + dc * 8);
    const float p = sc[j];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(p, bf2f(t.v[e]), acc[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o2 = 32; o2 >= 8; o2 >>= 1) acc[e] += __shfl_xor(acc[e], o2, 64);
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) oacc[wid * 64 + dc * 8 + e] = acc[e];
  }
  __syncthreads();
  if (tid < 64) {
    const float r = (oacc[tid] + oacc[64 + tid] + oacc[128 + tid] + oacc[192 + tid]) * inv;
    o[(size_t)b * H + head * 64 + tid] = f2bf(r);
  }
}

// h[b][r] += bf16(x[b] . W[r]) for the 16 rows of this workgroup (4 per wave, R rows total).
template <int B>
__global__ __launch_bounds__(DEC_NT) void k_dec_gemv_res(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                         float* __restrict__ h, int R, int K) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(dsm);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 16 + wid * 4;
  const bf16_t* rows[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rows[r] = w + (size_t)min(r0 + r, R - 1) * K;
  RowsPre<4, 4> pre;
  rows_pre<4, 4>(rows, K, pre);
  stage_copy<B>(x, K, xs);
  float acc[4][B];
  rows_dot<B, 4, 4>(rows, K, xs, pre, acc);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r0 + r < R) {
#pragma unroll
        for (int b = 0; b < B; ++b) h[(size_t)b * R + r0 + r] += bf_round(acc[r][b]);
      }
  }
}

// s[b][i] = bf16(silu(g) * u), g = bf16(n2 . Wgu[i]), u = bf16(n2 . Wgu[I + i]); 8 columns
// per workgroup, 2 per wave (4 rows: gate, up of each).
template <int B>
__global__ __launch_bounds__(DEC_NT) void k_dec_norm_gu(const float* __restrict__ h, const void* __restrict__ lnw,
                                                        int wbf16, float eps, const bf16_t* __restrict__ wgu,
                                                        bf16_t* __restrict__ s, int H, int I) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(dsm);
  float* red = reinterpret_cast<float*>(dsm + (size_t)B * H * 2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i0 = blockIdx.x * 8 + wid * 2;
  const int ia = min(i0, I - 1), ib = min(i0 + 1, I - 1);
  const bf16_t* rows[4] = {wgu + (size_t)ia * H, wgu + (size_t)(I + ia) * H, wgu + (size_t)ib * H,
                           wgu + (size_t)(I + ib) * H};
  RowsPre<4, 2> pre;
  rows_pre<4, 2>(rows, H, pre);
  stage_normed<B>(h, H, lnw, wbf16, eps, xs, red);
  float acc[4][B];
  rows_dot<B, 4, 2>(rows, H, xs, pre, acc);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (i0 + c < I) {
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const float gb = bf_round(acc[2 * c][b]), ub = bf_round(acc[2 * c + 1][b]);
          s[(size_t)b * I + i0 + c] = f2bf(gb * dlt_sigmoid(gb) * ub);
        }
      }
  }
}

// logits[b][r] = float(bf16(RMSNorm(h[b]) . E[r])) for r < V; 16 rows per workgroup.
template <int B>
__global__ __launch_bounds__(DEC_NT) void k_dec_norm_head(const float* __restrict__ h, const void* __restrict__ lnw,
                                                          int wbf16, float eps, const bf16_t* __restrict__ emb,
                                                          float* __restrict__ logits, int H, int V) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(dsm);
  float* red = reinterpret_cast<float*>(dsm + (size_t)B * H * 2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 16 + wid * 4;
  const bf16_t* rows[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rows[r] = emb + (size_t)min(r0 + r, V - 1) * H;
  RowsPre<4, 2> pre;
  rows_pre<4, 2>(rows, H, pre);
  stage_normed<B>(h, H, lnw, wbf16, eps, xs, red);
  float acc[4][B];
  rows_dot<B, 4, 2>(rows, H, xs, pre, acc);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r0 + r < V) {
#pragma unroll
        for (int b = 0; b < B; ++b) logits[(size_t)b * V + r0 + r] = bf_round(acc[r][b]);
      }
  }
}

// ---------------------------------------------------------------- top-k sampling
// GPT.generate's sampling step (gpt.py:474-482): logits / temperature, keep the values >=
// the k-th largest (ties kept, as masked_fill(lg < v[:, [-1]], -inf) does), softmax,
// one multinomial draw -- one row per workgroup of 512 threads (the row is re-read from L2
// by every pass: ~200 KB per row).  The k-th largest is found by a
// radix select on order-preserving uint32 keys (12 + 12 + 8 bits, LDS histograms, block
// suffix scans); the draw inverts the cumulative sum of exp(x - max) over the kept values
// with a counter-hash uniform of (seed, position, row).  The sampled id
// is written into the next step's input and into the generated-token history, so the
// whole generate loop runs on the device (one graph replay per token).
constexpr int SMP_NT = 512;

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// exclusive prefix sum over the block (SMP_NT threads) of v; returns it, total in *tot
__device__ __forceinline__ float block_excl_scan(float v, float* scr, float* tot) {
  constexpr int NW = SMP_NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) scr[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    float a = 0.f;
    for (int w = 0; w < NW; ++w) {  // inclusive per-wave prefix
      a += scr[w];
      scr[16 + w] = a;
    }
  }
  __syncthreads();
  const float base = wid ? scr[16 + wid - 1] : 0.f;
  *tot = scr[16 + NW - 1];
  __syncthreads();
  return base + incl - v;
}

// The k-th largest key of the row (k >= 1): radix select over bit fields [31:20], [19:8],
// [7:0]; key_at(j) returns this thread's j-th key (j < C), re-read from L2 each pass.
template <typename KeyAt>
__device__ uint32_t kth_key(KeyAt key_at, int C, int k, uint32_t* hist, float* scr, int* sel) {
  const int tid = threadIdx.x;
  uint32_t prefix = 0, pmask = 0;
  const int shifts[3] = {20, 8, 0}, widths[3] = {12, 12, 8};
#pragma unroll
  for (int ps = 0; ps < 3; ++ps) {
    const int sh = shifts[ps], nb = 1 << widths[ps];
    for (int i = tid; i < nb; i += SMP_NT) hist[i] = 0;
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < C; ++j) {
      const uint32_t kj = key_at(j);
      if ((kj & pmask) == prefix) atomicAdd(&hist[(kj >> sh) & (nb - 1)], 1u);
    }
    __syncthreads();
    // counts in descending-bin order: thread t owns reversed bins [8t, 8t + 8)
    float c[8], own = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = 8 * tid + q;
      c[q] = r < nb ? (float)hist[nb - 1 - r] : 0.f;
      own += c[q];
    }
    float total;
    float before = block_excl_scan(own, scr, &total);  // keys in higher bins than this thread's
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = 8 * tid + q;
      if (r < nb && before < (float)k && (float)k <= before + c[q]) {
        sel[0] = nb - 1 - r;
        sel[1] = k - (int)before;
      }
      before += c[q];
    }
    __syncthreads();
    prefix |= (uint32_t)sel[0] << sh;
    pmask |= (uint32_t)(nb - 1) << sh;
    k = sel[1];
    __syncthreads();
  }
  return prefix;
}

__device__ void sample_row(const float* __restrict__ logits, int V, float temperature, int top_k, uint32_t seed,
                           const long* __restrict__ posp, long* __restrict__ ids, long* __restrict__ hist,
                           int hist_len, int hist_base, int b, uint32_t* bins, float* scr, int* sel) {
  const int tid = threadIdx.x;
  // Thread t owns the elements i = t + SMP_NT * j (coalesced loads).  The draw inverts the
  // cumulative sum in (thread, j) order -- any fixed order of the elements samples the
  // same distribution.
  const int C = (V + SMP_NT - 1) / SMP_NT;
  const float* row = logits + (size_t)b * V;
  auto idx_of = [&](int j) { return tid + SMP_NT * j; };
  auto x_at = [&](int j) { const int i = idx_of(j); return i < V ? row[i] / temperature : -INFINITY; };
  auto key_at = [&](int j) { return f2key(x_at(j)); };
  float mx = -INFINITY;
#pragma unroll 4
  for (int j = 0; j < C; ++j) mx = fmaxf(mx, x_at(j));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) scr[tid >> 6] = mx;
  __syncthreads();
  mx = scr[0];
  for (int w = 1; w < SMP_NT / 64; ++w) mx = fmaxf(mx, scr[w]);
  __syncthreads();
  uint32_t thr = f2key(-INFINITY) + 1;  // keep every finite value
  if (top_k > 0 && top_k < V) {
    // Fast path: bracket the k-th largest with a value window below the max (count-only
    // passes, no atomics), collect the <= NCAND candidates into LDS and rank them there.
    // The radix select (LDS histograms) is the fallback for flat / tied distributions.
    constexpr int NCAND = 1024;
    uint32_t* cand = bins;  // reuse the histogram LDS
    float d = 4.f;
    int cnt = 0;
    bool ok = false;
    for (int it = 0; it < 8 && !ok; ++it) {
      const float t = mx - d;
      float own_c = 0.f;
#pragma unroll 4
      for (int j = 0; j < C; ++j) own_c += x_at(j) >= t ? 1.f : 0.f;
      float tot;
      (void)block_excl_scan(own_c, scr, &tot);
      cnt = (int)tot;
      if (cnt < top_k) d *= 2.f;
      else if (cnt > NCAND) d *= 0.5f;
      else ok = true;
    }
    if (ok) {
      const float t = mx - d;
      if (tid == 0) sel[0] = 0;
      __syncthreads();
#pragma unroll 4
      for (int j = 0; j < C; ++j) {
        const float x = x_at(j);
        if (x >= t) cand[atomicAdd(&sel[0], 1)] = f2key(x);
      }
      __syncthreads();
      // rank: the k-th largest candidate c has #{> c} < k <= #{>= c}
      for (int i = tid; i < cnt; i += SMP_NT) {
        const uint32_t ci = cand[i];
        int gt = 0, ge = 0;
        for (int m = 0; m < cnt; ++m) {
          const uint32_t cm = cand[m];
          gt += cm > ci;
          ge += cm >= ci;
        }
        if (gt < top_k && top_k <= ge) sel[1] = (int)ci;
      }
      __syncthreads();
      thr = max(thr, (uint32_t)sel[1]);
      __syncthreads();
    } else {
      thr = max(thr, kth_key(key_at, C, top_k, bins, scr, sel));
    }
  }
  float own = 0.f;
#pragma unroll 4
  for (int j = 0; j < C; ++j) {
    const float x = x_at(j);
    if (f2key(x) >= thr) own += __expf(x - mx);
  }
  float total;
  const float before = block_excl_scan(own, scr, &total);
  const long pos = posp[0];
  const uint32_t h = lowbias32(seed ^ lowbias32((uint32_t)pos * 0x9E3779B9u + (uint32_t)b));
  const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f) * total;  // (0, total)
  if (tid == 0) sel[0] = -1;
  __syncthreads();
  if (own > 0.f && before <= u && u < before + own) {
    float cum = before;
    int pick = -1, last = -1;
    for (int j = 0; j < C; ++j) {
      const float x = x_at(j);
      if (f2key(x) >= thr) {
        cum += __expf(x - mx);
        last = idx_of(j);
        if (u < cum) {
          pick = idx_of(j);
          break;
        }
      }
    }
    sel[0] = pick >= 0 ? pick : last;  // rounding at the slice end: its last kept value
  }
  __syncthreads();
  if (tid == 0) {
    int pick = sel[0];
    if (pick < 0) pick = 0;  // unreachable unless every probability underflowed
    ids[b] = pick;
    const long t = pos + 1 - hist_base;  // the token that will sit at position pos + 1
    if (t >= 0 && t < hist_len) hist[(size_t)b * hist_len + t] = pick;
  }
}

__global__ __launch_bounds__(SMP_NT) void k_dec_sample(const float* __restrict__ logits, int V, float temperature,
                                                       int top_k, uint32_t seed, const long* __restrict__ posp,
                                                       long* __restrict__ ids, long* __restrict__ hist, int hist_len,
                                                       int hist_base) {
  __shared__ uint32_t bins[4096];
  __shared__ float scr[40];
  __shared__ int sel[2];
  sample_row(logits, V, temperature, top_k, seed, posp, ids, hist, hist_len, hist_base, blockIdx.x, bins, scr, sel);
}

// Split sampler for 1 <= top_k <= 64: SMP_NS workgroups per row each take a slice of the
// row into LDS and keep its elements >= the slice's own k-th largest (ties included, at
// most SMP_MAXC: an element of the global top-k ranks within the top-k of its slice, so
// the union holds every kept element); one workgroup per row then ranks the <= 2048
// candidates and draws.  A slice that overflows SMP_MAXC sends its row to sample_row().
constexpr int SMP_NS = 16, SMP_MAXC = 128, SMP_SLICE = 4096;

__global__ __launch_bounds__(SMP_NT) void k_dec_topk_slices(const float* __restrict__ logits, int V,
                                                            float temperature, int top_k, int* __restrict__ ws) {
  __shared__ uint32_t keys[SMP_SLICE];
  __shared__ uint32_t bins[4096];
  __shared__ float scr[40];
  __shared__ int sel[2];
  const int tid = threadIdx.x, sl = blockIdx.x, b = blockIdx.y;
  const int L = (V + SMP_NS - 1) / SMP_NS, lo = sl * L, n = max(0, min(V, lo + L) - lo);
  const float* row = logits + (size_t)b * V + lo;
  uint32_t kmax = 0;
  for (int i = tid; i < SMP_SLICE; i += SMP_NT) {
    const uint32_t k = i < n ? f2key(row[i] / temperature) : 0u;  // 0: below every real key
    keys[i] = k;
    kmax = max(kmax, k);
  }
  __syncthreads();
  // ws row layout (ints): [SMP_NS] counts | [SMP_NS] max keys | [SMP_NS][SMP_MAXC] keys | idx
  int* cnt = ws + (size_t)b * SMP_NS * (2 + 2 * SMP_MAXC);
  int* maxk = cnt + SMP_NS;
  int* ck = maxk + SMP_NS + sl * SMP_MAXC;
  int* ci = maxk + SMP_NS + SMP_NS * SMP_MAXC + sl * SMP_MAXC;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
  if ((tid & 63) == 0) bins[tid >> 6] = kmax;
  __syncthreads();
  if (tid == 0) {
    uint32_t m = 0;
    for (int w = 0; w < SMP_NT / 64; ++w) m = max(m, bins[w]);
    maxk[sl] = (int)m;
  }
  __syncthreads();
  uint32_t lt = 1;  // keep every real element of a short slice
  if (top_k < n) {
    auto key_at = [&](int j) { return keys[tid + SMP_NT * j]; };
    lt = max(lt, kth_key(key_at, SMP_SLICE / SMP_NT, top_k, bins, scr, sel));
  }
  if (tid == 0) sel[0] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += SMP_NT) {
    const uint32_t k = keys[i];
    if (k >= lt) {
      const int slot = atomicAdd(&sel[0], 1);
      if (slot < SMP_MAXC) {
        ck[slot] = (int)k;
        ci[slot] = lo + i;
      }
    }
  }
  __syncthreads();
  if (tid == 0) cnt[sl] = sel[0] <= SMP_MAXC ? sel[0] : -1;  // -1: overflow
}

__global__ __launch_bounds__(SMP_NT) void k_dec_topk_draw(const int* __restrict__ ws, const float* __restrict__ logits,
                                                          int V, float temperature, int top_k, uint32_t seed,
                                                          const long* __restrict__ posp, long* __restrict__ ids,
                                                          long* __restrict__ hist, int hist_len, int hist_base) {
  __shared__ uint32_t ckey[SMP_NS * SMP_MAXC];
  __shared__ int cidx[SMP_NS * SMP_MAXC];
  __shared__ uint32_t bins[4096];
  __shared__ float scr[40];
  __shared__ int sel[2];
  const int tid = threadIdx.x, b = blockIdx.x;
  const int* cnt = ws + (size_t)b * SMP_NS * (2 + 2 * SMP_MAXC);
  const int* maxk = cnt + SMP_NS;
  const int* ck = maxk + SMP_NS;
  const int* ci = ck + SMP_NS * SMP_MAXC;
  bool overflow = false;
  uint32_t kmax = 0;
  for (int sl = 0; sl < SMP_NS; ++sl) {
    overflow |= cnt[sl] < 0;
    kmax = max(kmax, (uint32_t)maxk[sl]);
  }
  if (overflow) {  // (uniform) a slice had more than SMP_MAXC elements tied at its threshold
    sample_row(logits, V, temperature, top_k, seed, posp, ids, hist, hist_len, hist_base, b, bins, scr, sel);
    return;
  }
  for (int i = tid; i < SMP_NS * SMP_MAXC; i += SMP_NT) {
    const int sl = i / SMP_MAXC, j = i - sl * SMP_MAXC;
    const bool ok = j < cnt[sl];
    ckey[i] = ok ? (uint32_t)ck[i] : 0u;
    cidx[i] = ok ? ci[i] : -1;
  }
  __syncthreads();
  constexpr int PT = SMP_NS * SMP_MAXC / SMP_NT;  // candidates per thread: tid + SMP_NT * j
  auto key_at = [&](int j) { return ckey[tid + SMP_NT * j]; };
  const uint32_t thr = max(1u, kth_key(key_at, PT, top_k, bins, scr, sel));
  const float mx = key2f(kmax);
  float own = 0.f;
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const uint32_t k = key_at(j);
    if (k >= thr) own += __expf(key2f(k) - mx);
  }
  float total;
  const float before = block_excl_scan(own, scr, &total);
  const long pos = posp[0];
  const uint32_t h = lowbias32(seed ^ lowbias32((uint32_t)pos * 0x9E3779B9u + (uint32_t)b));
  const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f) * total;
  if (tid == 0) sel[0] = -1;
  __syncthreads();
  if (own > 0.f && before <= u && u < before + own) {
    float cum = before;
    int pick = -1, last = -1;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const uint32_t k = key_at(j);
      if (k >= thr) {
        cum += __expf(key2f(k) - mx);
        last = cidx[tid + SMP_NT * j];
        if (pick < 0 && u < cum) pick = last;
      }
    }
    sel[0] = pick >= 0 ? pick : last;
  }
  __syncthreads();
  if (tid == 0) {
    const int pick = sel[0] < 0 ? 0 : sel[0];
    ids[b] = pick;
    const long t = pos + 1 - hist_base;
    if (t >= 0 && t < hist_len) hist[(size_t)b * hist_len + t] = pick;
  }
}

__global__ void k_dec_advance(long* pos) { pos[0] += 1; }

// ------------------------------------------------------------------------ launchers
#define DEC_DISPATCH(B, CALL)          \
  switch (B) {                         \
    case 1: CALL(1); break;            \
    case 2: CALL(2); break;            \
    case 4: CALL(4); break;            \
    case 8: CALL(8); break;            \
    default: return -1;                \
  }

static size_t dec_lds(int B, int K) { return (size_t)B * K * 2 + (size_t)B * 4 * 4 + (size_t)B * 16 * 4; }

DLT_API int dlt_dec_norm_qkv(const float* h, const void* lnw, int wbf16, float eps, const bf16_t* wqkv,
                             const float* cosT, const float* sinT, const long* pos, bf16_t* qout, bf16_t* kc,
                             bf16_t* vc, int B, int H, int nh, int maxS, hipStream_t st) {
  if (H != nh * 64 || H % 8 || dec_lds(B, H) > 160 * 1024) return -1;
#define L(BB)                                                                                                      \
  k_dec_norm_qkv<BB><<<3 * nh * 4, DEC_NT, dec_lds(BB, H), st>>>(h, lnw, wbf16, eps, wqkv, cosT, sinT, pos, qout, kc, vc, \
                                                             H, nh, maxS)
  DEC_DISPATCH(B, L)
#undef L
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_dec_attn(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const long* pos, bf16_t* o, int B,
                         int H, int nh, int maxS, float scale, hipStream_t st) {
  const size_t lds = (size_t)maxS * 4 + 8 * 4 + 4 * 64 * 4;
  if (H != nh * 64 || lds > 160 * 1024) return -1;
  k_dec_attn<<<B * nh, DEC_NT, lds, st>>>(q, kc, vc, pos, o, H, nh, maxS, scale);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_dec_gemv_res(const bf16_t* x, const bf16_t* w, float* h, int B, int R, int K, hipStream_t st) {
  if (K % 8 || (size_t)B * K * 2 > 160 * 1024) return -1;
#define L(BB) k_dec_gemv_res<BB><<<(R + 15) / 16, DEC_NT, (size_t)BB * K * 2, st>>>(x, w, h, R, K)
  DEC_DISPATCH(B, L)
#undef L
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_dec_norm_gu(const float* h, const void* lnw, int wbf16, float eps, const bf16_t* wgu, bf16_t* s,
                            int B, int H, int I, hipStream_t st) {
  if (H % 8 || dec_lds(B, H) > 160 * 1024) return -1;
#define L(BB) k_dec_norm_gu<BB><<<(I + 7) / 8, DEC_NT, dec_lds(BB, H), st>>>(h, lnw, wbf16, eps, wgu, s, H, I)
  DEC_DISPATCH(B, L)
#undef L
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_dec_norm_head(const float* h, const void* lnw, int wbf16, float eps, const bf16_t* emb,
                              float* logits, int B, int H, int V, hipStream_t st) {
  if (H % 8 || dec_lds(B, H) > 160 * 1024) return -1;
#define L(BB) k_dec_norm_head<BB><<<(V + 15) / 16, DEC_NT, dec_lds(BB, H), st>>>(h, lnw, wbf16, eps, emb, logits, H, V)
  DEC_DISPATCH(B, L)
#undef L
  DLT_CHECK_LAUNCH();
}

// ids [B] (int64, the next step's input), hist [B, hist_len]: hist[b][pos + 1 - hist_base] = sampled id
// ws: int32 workspace of B * 16 * 258 (dlt_dec_sample_ws_ints); nullptr -> one workgroup per row
DLT_API int dlt_dec_sample_ws_ints(int B) { return B * SMP_NS * (2 + 2 * SMP_MAXC); }
DLT_API int dlt_dec_sample(const float* logits, int B, int V, float temperature, int top_k, uint32_t seed,
                           const long* pos, long* ids, long* hist, int hist_len, int hist_base, int* ws,
                           hipStream_t st) {
  if (V <= 0 || temperature <= 0.f) return -1;
  if (ws && top_k >= 1 && top_k <= 64 && V <= SMP_NS * SMP_SLICE && top_k < V) {
    k_dec_topk_slices<<<dim3(SMP_NS, B), SMP_NT, 0, st>>>(logits, V, temperature, top_k, ws);
    k_dec_topk_draw<<<B, SMP_NT, 0, st>>>(ws, logits, V, temperature, top_k, seed, pos, ids, hist, hist_len,
                                          hist_base);
  } else {
    k_dec_sample<<<B, SMP_NT, 0, st>>>(logits, V, temperature, top_k, seed, pos, ids, hist, hist_len, hist_base);
  }
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_dec_advance(long* pos, hipStream_t st) {
  k_dec_advance<<<1, 1, 0, st>>>(pos);
  DLT_CHECK_LAUNCH();
}
