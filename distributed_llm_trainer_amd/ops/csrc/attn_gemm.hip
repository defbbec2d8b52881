// Attention as batched GEMMs: the row kernels between the products, and the layout copy
// that feeds them (ops/hip_f32.py: fp32 activations; ops/attn_gemm.py: head dims without a
// flash kernel, in any precision).
//
// The six S x S x hd products run as batched hipBLASLt GEMMs over the dense [S, S] score
// matrix of every (b, h): Q·Kᵀ, P·V forward and Q·Kᵀ, dO·Vᵀ, Pdᵀ·dO, dS·K, dSᵀ·Q backward.
// The scores and dO·Vᵀ always come out in fp32.  The operands the kernels below write
// are P, Pd and dS.  They are in the activation format OT: 0 = fp32 (in place over the
// scores), 1 = bf16, 2 = fp16 (separate buffers).  So 16-bit runs keep the flash kernels'
// arithmetic: fp32 scores and softmax, P and dS rounded to 16 bits as MFMA operands.
//
//   * k_attn_softmax<NE, OT>   -- causal mask, softmax, lse (natural log) and dropout from
//     the keep-bit words of k_dropout_bits (attention.hip), one 256-thread block per row;
//     k_attn_softmax_w / k_attn_dsoftmax_w: one wave per row, 4 rows per workgroup, float4
//     score accesses and wave-only reductions (no LDS, no barrier), for S % 4 == 0;
//     k_attn_softmax_long: rows of more than 4096 keys (three passes over the row)
//   * k_attn_dsoftmax<OT>      -- P from lse, delta = rowsum(dO * O), the dropped P (for
//     dV) and scale * dS (for dQ / dK)
//   * k_relayout16             -- 16-bit [b, s, h, d] strided copy (packed QKV <-> head-major)
#include "common.h"

namespace {

template <int OT>
struct ATy {
  using T = uint16_t;
};
template <>
struct ATy<0> {
  using T = float;
};

template <int OT>
__device__ __forceinline__ float a_ld(const typename ATy<OT>::T* p, size_t i) {
  if constexpr (OT == 0) return p[i];
  else return h2f<OT - 1>(p[i]);
}

template <int OT>
__device__ __forceinline__ void a_st(typename ATy<OT>::T* p, size_t i, float v) {
  if constexpr (OT == 0) p[i] = v;
  else p[i] = f2h<OT - 1>(v);
}

__device__ __forceinline__ float ag_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float ag_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide max / sum over the 4 waves, returned to every thread
template <bool MAX>
__device__ __forceinline__ float ag_block_reduce(float v, float* red) {
  v = MAX ? ag_wave_max(v) : ag_wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = MAX ? fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])) : (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();  // red is reused by the next reduction
  return r;
}

}  // namespace

// sc [BH*S, S] raw scores q·k (fp32) -> pout [BH*S, S] = keep * dscale * softmax(scale * s)
// over keys <= q (zeros after q), lse [BH*S].  NE keys per thread (S <= 256 * NE).  OT = 0:
// pout may be sc (every score is in registers before the first store).
template <int NE, int OT>
__global__ __launch_bounds__(256) void k_attn_softmax(const float* sc, typename ATy<OT>::T* pout,
                                                      float* __restrict__ lse, const uint32_t* __restrict__ mask,
                                                      int S, float scale, float dscale, int Lb) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const int q = (int)(row % S);
  const long bh = row / S;
  const int wl = Lb > 0 ? min(S, (q / Lb + 1) * Lb) : S;  // columns the blocked GEMMs read
  const float* r = sc + row * S;
  const float c = scale * 1.44269504088896341f;
  float x[NE];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int k = threadIdx.x + 256 * i;
    x[i] = k <= q ? r[k] * c : -INFINITY;
    m = fmaxf(m, x[i]);
  }
  m = ag_block_reduce<true>(m, red);  // finite: key 0 is always visible
  float l = 0.f;
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    x[i] = exp2f(x[i] - m);
    l += x[i];
  }
  l = ag_block_reduce<false>(l, red);
  if (threadIdx.x == 0) lse[row] = (m + __log2f(l)) * 0.69314718055994531f;
  const float inv = 1.f / l;
  const uint32_t* mw = mask ? mask + bh * (long)((S + 31) >> 5) * S + q : nullptr;
  typename ATy<OT>::T* po = pout + row * S;
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int k = threadIdx.x + 256 * i;
    if (k >= wl) break;
    float p = 0.f;
    if (k <= q) {
      p = x[i] * inv;
      if (mw) p = ((mw[(size_t)(k >> 5) * S] >> (k & 31)) & 1u) ? p * dscale : 0.f;
    }
    a_st<OT>(po, k, p);
  }
}

// Per (bh, q) row: sc = recomputed scores q·k, dp = dO·vᵀ (fp32, the gradient of the
// dropped probabilities).  Writes pd = the dropped probabilities (for dV = Pdᵀ·dO) and
// ds = scale * p * (keep * dscale * dp - delta) (for dQ = dS·K, dK = dSᵀ·Q); delta =
// rowsum(dO * O) from o / dO [B*S, nh*hd] in the activation format.  OT = 0: pd / ds may
// be sc / dp (element-wise in place).
template <int OT>
__global__ __launch_bounds__(256) void k_attn_dsoftmax(const float* sc, const float* dp, typename ATy<OT>::T* pd_out,
                                                       typename ATy<OT>::T* ds_out, const float* __restrict__ lse,
                                                       const typename ATy<OT>::T* __restrict__ o,
                                                       const typename ATy<OT>::T* __restrict__ dO,
                                                       const uint32_t* __restrict__ mask, int S, int nh, int hd,
                                                       float scale, float dscale, int Lb) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const int q = (int)(row % S);
  const long bh = row / S;
  const long b = bh / nh, h = bh % nh;
  const size_t orow = ((size_t)(b * S + q) * nh + h) * hd;
  float dl = 0.f;
  for (int d = threadIdx.x; d < hd; d += 256) dl = fmaf(a_ld<OT>(o, orow + d), a_ld<OT>(dO, orow + d), dl);
  const float delta = ag_block_reduce<false>(dl, red);
  const float ls = lse[row];
  const float* rs = sc + row * S;
  const float* rd = dp + row * S;
  typename ATy<OT>::T* wp = pd_out + row * S;
  typename ATy<OT>::T* wd = ds_out + row * S;
  const uint32_t* mw = mask ? mask + bh * (long)((S + 31) >> 5) * S + q : nullptr;
  const int wl = Lb > 0 ? min(S, (q / Lb + 1) * Lb) : S;
  for (int k = threadIdx.x; k < wl; k += 256) {
    float pd = 0.f, ds = 0.f;
    if (k <= q) {
      const float p = __expf(rs[k] * scale - ls);
      float g = rd[k];
      pd = p;
      if (mw) {
        const bool keep = (mw[(size_t)(k >> 5) * S] >> (k & 31)) & 1u;
        pd = keep ? p * dscale : 0.f;
        g = keep ? g * dscale : 0.f;
      }
      ds = p * (g - delta) * scale;
    }
    a_st<OT>(wp, k, pd);
    a_st<OT>(wd, k, ds);
  }
}

// 4 consecutive values at p (float4 for fp32, one 8-byte store for 16-bit)
template <int OT>
__device__ __forceinline__ void a_st4(typename ATy<OT>::T* p, const float (&v)[4]) {
  if constexpr (OT == 0) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 w;
    w.x = (uint32_t)f2h<OT - 1>(v[0]) | ((uint32_t)f2h<OT - 1>(v[1]) << 16);
    w.y = (uint32_t)f2h<OT - 1>(v[2]) | ((uint32_t)f2h<OT - 1>(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = w;
  }
}

// k_attn_softmax with one wave per row: lane l owns columns 4l + 256i (i < NV, S <= 256 NV,
// S % 4 == 0); the 4 columns of a group share one keep-bit word.
template <int NV, int OT>
__global__ __launch_bounds__(256) void k_attn_softmax_w(const float* sc, typename ATy<OT>::T* pout,
                                                        float* __restrict__ lse, const uint32_t* __restrict__ mask,
                                                        long rows, int S, float scale, float dscale, int Lb) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int q = (int)(row % S);
  const long bh = row / S;
  const float* r = sc + row * S;
  const float c = scale * 1.44269504088896341f;
  float x[NV][4];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c0 = 4 * lane + 256 * i;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c0 <= q) v = *reinterpret_cast<const float4*>(r + c0);  // c0 <= q < S: the group is in the row
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[i][e] = c0 + e <= q ? vv[e] * c : -INFINITY;
      m = fmaxf(m, x[i][e]);
    }
  }
  m = wave_max(m);  // finite: key 0 is always visible
  float l = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[i][e] = exp2f(x[i][e] - m);
      l += x[i][e];
    }
  l = wave_sum(l);
  if (lane == 0) lse[row] = (m + __log2f(l)) * 0.69314718055994531f;
  const float inv = 1.f / l;
  const uint32_t* mw = mask ? mask + bh * (long)((S + 31) >> 5) * S + q : nullptr;
  typename ATy<OT>::T* po = pout + row * S;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c0 = 4 * lane + 256 * i;
    if (c0 >= (Lb > 0 ? min(S, (q / Lb + 1) * Lb) : S)) break;
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    if (c0 <= q) {
      const uint32_t w = mw ? mw[(size_t)(c0 >> 5) * S] >> (c0 & 31) : ~0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pe = x[i][e] * inv;
        p[e] = mw ? (((w >> e) & 1u) ? pe * dscale : 0.f) : pe;
      }
    }
    a_st4<OT>(po + c0, p);
  }
}

// k_attn_softmax for rows longer than the register-resident kernels above take (S > 4096
// keys): one wave per row, three passes over the row in memory (max, sum, write), the same
// arithmetic.  OT = 0: pout may be sc (each element is read and written by one lane).
template <int OT>
__global__ __launch_bounds__(256) void k_attn_softmax_long(const float* sc, typename ATy<OT>::T* pout,
                                                           float* __restrict__ lse, const uint32_t* __restrict__ mask,
                                                           long rows, int S, float scale, float dscale, int Lb) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int q = (int)(row % S);
  const long bh = row / S;
  const float* r = sc + row * S;
  const float c = scale * 1.44269504088896341f;
  float m = -INFINITY;
  for (int k = lane; k <= q; k += 64) m = fmaxf(m, r[k] * c);
  m = wave_max(m);  // finite: key 0 is always visible
  float l = 0.f;
  for (int k = lane; k <= q; k += 64) l += exp2f(r[k] * c - m);
  l = wave_sum(l);
  if (lane == 0) lse[row] = (m + __log2f(l)) * 0.69314718055994531f;
  const float inv = 1.f / l;
  const uint32_t* mw = mask ? mask + bh * (long)((S + 31) >> 5) * S + q : nullptr;
  typename ATy<OT>::T* po = pout + row * S;
  const int wl = Lb > 0 ? min(S, (q / Lb + 1) * Lb) : S;
  for (int k = lane; k < wl; k += 64) {
    float p = 0.f;
    if (k <= q) {
      p = exp2f(r[k] * c - m) * inv;
      if (mw) p = ((mw[(size_t)(k >> 5) * S] >> (k & 31)) & 1u) ? p * dscale : 0.f;
    }
    a_st<OT>(po, k, p);
  }
}

// k_attn_dsoftmax with one wave per row (S % 4 == 0)
template <int OT>
__global__ __launch_bounds__(256) void k_attn_dsoftmax_w(const float* sc, const float* dp, typename ATy<OT>::T* pd_out,
                                                         typename ATy<OT>::T* ds_out, const float* __restrict__ lse,
                                                         const typename ATy<OT>::T* __restrict__ o,
                                                         const typename ATy<OT>::T* __restrict__ dO,
                                                         const uint32_t* __restrict__ mask, long rows, int S, int nh,
                                                         int hd, float scale, float dscale, int Lb) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int q = (int)(row % S);
  const long bh = row / S;
  const long b = bh / nh, h = bh % nh;
  const size_t orow = ((size_t)(b * S + q) * nh + h) * hd;
  float dl = 0.f;
  for (int d = lane; d < hd; d += 64) dl = fmaf(a_ld<OT>(o, orow + d), a_ld<OT>(dO, orow + d), dl);
  const float delta = wave_sum(dl);
  const float ls = lse[row];
  const float* rs = sc + row * S;
  const float* rd = dp + row * S;
  typename ATy<OT>::T* wp = pd_out + row * S;
  typename ATy<OT>::T* wd = ds_out + row * S;
  const uint32_t* mw = mask ? mask + bh * (long)((S + 31) >> 5) * S + q : nullptr;
  const int wl = Lb > 0 ? min(S, (q / Lb + 1) * Lb) : S;
  for (int c0 = 4 * lane; c0 < wl; c0 += 256) {
    float pd[4] = {0.f, 0.f, 0.f, 0.f}, ds[4] = {0.f, 0.f, 0.f, 0.f};
    if (c0 <= q) {
      const float4 s4 = *reinterpret_cast<const float4*>(rs + c0), g4 = *reinterpret_cast<const float4*>(rd + c0);
      const float sv[4] = {s4.x, s4.y, s4.z, s4.w}, gv[4] = {g4.x, g4.y, g4.z, g4.w};
      const uint32_t w = mw ? mw[(size_t)(c0 >> 5) * S] >> (c0 & 31) : ~0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (c0 + e > q) break;
        const float p = __expf(sv[e] * scale - ls);
        float g = gv[e];
        float pe = p;
        if (mw) {
          const bool keep = (w >> e) & 1u;
          pe = keep ? p * dscale : 0.f;
          g = keep ? g * dscale : 0.f;
        }
        pd[e] = pe;
        ds[e] = p * (g - delta) * scale;
      }
    }
    a_st4<OT>(wp + c0, pd);
    a_st4<OT>(wd + c0, ds);
  }
}

// 16-bit strided copy of ntens tensors: element (b, s, h, d) of tensor t at
// src + t*sts + b*sb + s*sr + h*sh + d -> dst + t*dts + b*db + s*dr + h*dh + d.  Grid x:
// (head, chunk of V elements) of a row, grid y strides over the B*S rows.  V = 8: 16-byte
// accesses (hd % 8 == 0 and every stride / base 16-byte aligned, checked by the launcher).
template <int V>
__global__ __launch_bounds__(256) void k_relayout16(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst, long sb,
                                                    long sr, long sh, long db, long dr, long dh, long sts, long dts,
                                                    int B, int S, int nh, int hd, int ntens) {
  const int per = hd / V;
  const int t0 = blockIdx.x * 256 + threadIdx.x;
  if (t0 >= nh * per) return;
  const int h = t0 / per, j = (t0 - h * per) * V;
  for (int r = blockIdx.y; r < B * S; r += gridDim.y) {
    const int b = r / S, s = r - b * S;
    const long so = b * sb + s * sr + h * sh + j, dof = b * db + s * dr + h * dh + j;
    for (int t = 0; t < ntens; ++t) {
      if constexpr (V == 8) {
        *reinterpret_cast<uint4*>(dst + t * dts + dof) = *reinterpret_cast<const uint4*>(src + t * sts + so);
      } else {
        dst[t * dts + dof] = src[t * sts + so];
      }
    }
  }
}

// DLT_ATTN_ROW_WAVE=0: the block-per-row kernels for every S (A/B)
static bool row_w_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DLT_ATTN_ROW_WAVE");
    v = (e && atoi(e) == 0) ? 0 : 1;
  }
  return v == 1;
}

template <int OT>
static int softmax_launch(float* sc, void* pout, float* lse, const uint32_t* mask, int BH, int S, float scale,
                          float dscale, int Lb, hipStream_t st) {
  const long rows = (long)BH * S;
  if (S <= 0 || rows > 0x7fffffffL || Lb < 0 || Lb % 4) return -1;
  using T = typename ATy<OT>::T;
  T* po = static_cast<T*>(pout);
  if (S > 4096) {  // rows longer than the register-resident kernels take
    k_attn_softmax_long<OT><<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(sc, po, lse, mask, rows, S, scale, dscale, Lb);
    return 0;
  }
  const int ne = (S + 255) / 256;
  if (S % 4 == 0 && row_w_enabled()) {  // wave per row (the 16-bit rows are 8-byte aligned: S % 4 == 0)
    const unsigned nb = (unsigned)((rows + 3) / 4);
    if (ne <= 1) k_attn_softmax_w<1, OT><<<nb, 256, 0, st>>>(sc, po, lse, mask, rows, S, scale, dscale, Lb);
    else if (ne <= 2) k_attn_softmax_w<2, OT><<<nb, 256, 0, st>>>(sc, po, lse, mask, rows, S, scale, dscale, Lb);
    else if (ne <= 4) k_attn_softmax_w<4, OT><<<nb, 256, 0, st>>>(sc, po, lse, mask, rows, S, scale, dscale, Lb);
    else if (ne <= 8) k_attn_softmax_w<8, OT><<<nb, 256, 0, st>>>(sc, po, lse, mask, rows, S, scale, dscale, Lb);
    else k_attn_softmax_w<16, OT><<<nb, 256, 0, st>>>(sc, po, lse, mask, rows, S, scale, dscale, Lb);
    return 0;
  }
  if (ne <= 1) k_attn_softmax<1, OT><<<rows, 256, 0, st>>>(sc, po, lse, mask, S, scale, dscale, Lb);
  else if (ne <= 2) k_attn_softmax<2, OT><<<rows, 256, 0, st>>>(sc, po, lse, mask, S, scale, dscale, Lb);
  else if (ne <= 4) k_attn_softmax<4, OT><<<rows, 256, 0, st>>>(sc, po, lse, mask, S, scale, dscale, Lb);
  else if (ne <= 8) k_attn_softmax<8, OT><<<rows, 256, 0, st>>>(sc, po, lse, mask, S, scale, dscale, Lb);
  else k_attn_softmax<16, OT><<<rows, 256, 0, st>>>(sc, po, lse, mask, S, scale, dscale, Lb);
  return 0;
}

template <int OT>
static int dsoftmax_launch(const float* sc, const float* dp, void* pd_out, void* ds_out, const float* lse,
                           const void* o, const void* dO, const uint32_t* mask, int B, int nh, int S, int hd,
                           float scale, float dscale, int Lb, hipStream_t st) {
  const long rows = (long)B * nh * S;
  if (S <= 0 || hd <= 0 || hd > 256 || rows > 0x7fffffffL || Lb < 0 || Lb % 4) return -1;
  using T = typename ATy<OT>::T;
  if (S % 4 == 0 && row_w_enabled()) {
    k_attn_dsoftmax_w<OT><<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(
        sc, dp, static_cast<T*>(pd_out), static_cast<T*>(ds_out), lse, static_cast<const T*>(o),
        static_cast<const T*>(dO), mask, rows, S, nh, hd, scale, dscale, Lb);
    return 0;
  }
  k_attn_dsoftmax<OT><<<rows, 256, 0, st>>>(sc, dp, static_cast<T*>(pd_out), static_cast<T*>(ds_out), lse,
                                            static_cast<const T*>(o), static_cast<const T*>(dO), mask, S, nh, hd, scale,
                                            dscale, Lb);
  return 0;
}

// Lb (every entry point): the row-block size of blocked causal GEMMs -- a row q only
// writes the columns below the end of its block, (q / Lb + 1) * Lb; 0: the whole row.
// fp32: sc [BH*S, S] in place; lse [BH*S]
DLT_API int dlt_f32_attn_softmax(float* sc, float* lse, const uint32_t* mask, int BH, int S, float scale, float dscale,
                                 int Lb, hipStream_t st) {
  if (softmax_launch<0>(sc, sc, lse, mask, BH, S, scale, dscale, Lb, st)) return -1;
  DLT_CHECK_LAUNCH();
}

// fp32: sc / dp [B*nh*S, S] in place; o / dO [B*S, nh*hd]
DLT_API int dlt_f32_attn_dsoftmax(float* sc, float* dp, const float* lse, const float* o, const float* dO,
                                  const uint32_t* mask, int B, int nh, int S, int hd, float scale, float dscale,
                                  int Lb, hipStream_t st) {
  if (dsoftmax_launch<0>(sc, dp, sc, dp, lse, o, dO, mask, B, nh, S, hd, scale, dscale, Lb, st)) return -1;
  DLT_CHECK_LAUNCH();
}

// 16-bit (hk 0 bf16, 1 fp16): fp32 scores sc -> P into pout [BH*S, S]
DLT_API int dlt_attn16_softmax(const float* sc, void* pout, float* lse, const uint32_t* mask, int BH, int S,
                               float scale, float dscale, int Lb, int hk, hipStream_t st) {
  const int rc = hk ? softmax_launch<2>(const_cast<float*>(sc), pout, lse, mask, BH, S, scale, dscale, Lb, st)
                    : softmax_launch<1>(const_cast<float*>(sc), pout, lse, mask, BH, S, scale, dscale, Lb, st);
  if (rc) return -1;
  DLT_CHECK_LAUNCH();
}

// 16-bit: fp32 sc / dp -> pd / ds [B*nh*S, S] (16-bit); o / dO [B*S, nh*hd] 16-bit
DLT_API int dlt_attn16_dsoftmax(const float* sc, const float* dp, void* pd_out, void* ds_out, const float* lse,
                                const void* o, const void* dO, const uint32_t* mask, int B, int nh, int S, int hd,
                                float scale, float dscale, int Lb, int hk, hipStream_t st) {
  const int rc = hk ? dsoftmax_launch<2>(sc, dp, pd_out, ds_out, lse, o, dO, mask, B, nh, S, hd, scale, dscale, Lb, st)
                    : dsoftmax_launch<1>(sc, dp, pd_out, ds_out, lse, o, dO, mask, B, nh, S, hd, scale, dscale, Lb, st);
  if (rc) return -1;
  DLT_CHECK_LAUNCH();
}

// strides in elements (see k_relayout16); ntens 1..3
DLT_API int dlt_relayout16(const uint16_t* src, uint16_t* dst, long sb, long sr, long sh, long db, long dr, long dh,
                           long sts, long dts, int B, int S, int nh, int hd, int ntens, hipStream_t st) {
  if (ntens < 1 || ntens > 3 || hd <= 0 || (long)B * S > 0x7fffffffL || B * S <= 0) return -1;
  const long al[] = {sb, sr, sh, db, dr, dh, sts, dts};
  bool v8 = hd % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0;
  for (long x : al) v8 = v8 && x % 8 == 0;
  const int per = v8 ? hd / 8 : hd;
  const dim3 grid((nh * per + 255) / 256, B * S < 65535 ? B * S : 65535);
  if (v8) k_relayout16<8><<<grid, 256, 0, st>>>(src, dst, sb, sr, sh, db, dr, dh, sts, dts, B, S, nh, hd, ntens);
  else k_relayout16<1><<<grid, 256, 0, st>>>(src, dst, sb, sr, sh, db, dr, dh, sts, dts, B, S, nh, hd, ntens);
  DLT_CHECK_LAUNCH();
}
