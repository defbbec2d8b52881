// Fused residual-add + dropout + RMSNorm (forward) and its backward.
//
// Replaces the reference's per-block sequence  x + dropout(f(x))  ->  RMSNorm
// (gpt.py:66, 240, 282, 308, 314: pow/mean/add/rsqrt/mul/mul + bernoulli + add =
// ~9 ATen kernels fwd, more bwd) with ONE memory pass each way:
//
//   fwd: x = resid + keep(delta)/(1-p);  y = bf16(x * rsqrt(mean(x^2)+eps) * w)
//   bwd: dx = dres + rstd*(g - xh*mean(g*xh)),  g = dy*w;  ddelta = keep(dx)/(1-p)
//        dw += sum_rows dy*xh
//
// One wave (64 lanes) owns one row; lane l holds the 4-element chunks l, l+64, ...
// in registers (NCH = ceil(H/256) chunks per lane; H = 768 -> exactly 3, every lane
// busy), so each tensor is touched once.  All loads of a row (dy, x, and the incoming
// residual gradient) are issued before the row reduction so their latencies overlap.
// The residual stream is fp32 (matches the reference DDP/autocast numerics, SURVEY
// §2.4 P9).
#include "common.h"
#include <cstdlib>

struct f4 { float v[4]; };

__device__ __forceinline__ f4 ld_f4(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  return f4{{a.x, a.y, a.z, a.w}};
}
__device__ __forceinline__ void st_f4(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <int HK>
__device__ __forceinline__ void ld_h4(const bf16_t* p, float (&v)[4]) {
  const u16x4 d = *reinterpret_cast<const u16x4*>(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = h2f<HK>(d.v[e]);
}

// Norm weight: fp32 (flat master, DDP path) or 16-bit in the activation format (the
// gathered FSDP unit) -- read in place, so the FSDP path needs no per-call weight upcast.
template <int HK>
__device__ __forceinline__ f4 ld_w4(const void* w, int w16, int off) {
  if (w16) {
    f4 r;
    ld_h4<HK>(reinterpret_cast<const bf16_t*>(w) + off, r.v);
    return r;
  }
  return ld_f4(reinterpret_cast<const float*>(w) + off);
}

__device__ __forceinline__ void st_f4_nt(float* p, const float (&v)[4]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) __builtin_nontemporal_store(v[e], p + e);
}

template <int NCH, bool XNT = false, int HK = 0>
__global__ __launch_bounds__(256) void k_add_dropout_rmsnorm_fwd(
    const float* __restrict__ resid, const bf16_t* __restrict__ delta, const void* __restrict__ w, int wbf16,
    float* __restrict__ x_out, bf16_t* __restrict__ y_out, float* __restrict__ rstd_out,
    int M, int H, float eps, uint32_t key, uint32_t thr, float dscale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nc = H >> 2;
  const size_t rbase = (size_t)row * H;
  float xv[NCH][4];
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < NCH; ++t) {
    const int c = lane + 64 * t;
#pragma unroll
    for (int e = 0; e < 4; ++e) xv[t][e] = 0.f;
    if (c < nc) {
      const size_t off = rbase + (size_t)c * 4;
      if (resid) {
        const f4 r = ld_f4(resid + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[t][e] = r.v[e];
      }
      if (delta) {
        float d[4];
        ld_h4<HK>(delta + off, d);
        if (thr) {
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const uint32_t h = lowbias32(key ^ (uint32_t)((off + e) >> 1));
            xv[t][e] += ((h & 0xffffu) >= thr) ? d[e] * dscale : 0.f;
            xv[t][e + 1] += ((h >> 16) >= thr) ? d[e + 1] * dscale : 0.f;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[t][e] += d[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) ss += xv[t][e] * xv[t][e];
    }
  }
  ss = wave_sum(ss);
  const float rstd = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd_out[row] = rstd;
#pragma unroll
  for (int t = 0; t < NCH; ++t) {
    const int c = lane + 64 * t;
    if (c < nc) {
      const size_t off = rbase + (size_t)c * 4;
      if (x_out) {  // the fp32 block input is read again only by the backward
        if (XNT) st_f4_nt(x_out + off, xv[t]);
        else st_f4(x_out + off, xv[t]);
      }
      const f4 ww = ld_w4<HK>(w, wbf16, c * 4);
      u16x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y.v[e] = f2h<HK>(xv[t][e] * rstd * ww.v[e]);
      *reinterpret_cast<u16x4*>(y_out + off) = y;
    }
  }
}

template <int NCH, int HK = 0>
__global__ __launch_bounds__(256) void k_rmsnorm_bwd(
    const bf16_t* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ rstd_in,
    const void* __restrict__ w, int wbf16, const float* dres, float* dx_out,
    bf16_t* __restrict__ ddelta, float* __restrict__ dw, float* __restrict__ dw_part,
    const float* __restrict__ dy_scale, float dy_mul, int M, int H, uint32_t key, uint32_t thr, float dscale) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [4][H]
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nc = H >> 2;
  const float sc = (dy_scale ? *dy_scale : 1.f) * dy_mul;
  const float invH = 1.f / (float)H;
  float dwacc[NCH][4];
  float wv[NCH][4];
#pragma unroll
  for (int t = 0; t < NCH; ++t) {
    const int c = lane + 64 * t;
#pragma unroll
    for (int e = 0; e < 4; ++e) { dwacc[t][e] = 0.f; wv[t][e] = 0.f; }
    if (c < nc) {
      const f4 a = ld_w4<HK>(w, wbf16, c * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) wv[t][e] = a.v[e];
    }
  }
  for (int row = blockIdx.x * 4 + wid; row < M; row += gridDim.x * 4) {
    const size_t rbase = (size_t)row * H;
    const float rstd = rstd_in[row];
    float dv[NCH][4], xx[NCH][4], rr[NCH][4];
    // issue every load of the row first
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
      const int c = lane + 64 * t;
#pragma unroll
      for (int e = 0; e < 4; ++e) { dv[t][e] = 0.f; xx[t][e] = 0.f; rr[t][e] = 0.f; }
      if (c < nc) {
        const size_t off = rbase + (size_t)c * 4;
        ld_h4<HK>(dy + off, dv[t]);
        const f4 a = ld_f4(x + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) xx[t][e] = a.v[e];
        if (dres) {
          const f4 r = ld_f4(dres + off);
#pragma unroll
          for (int e = 0; e < 4; ++e) rr[t][e] = r.v[e];
        }
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = dv[t][e] * sc;
        const float xh = xx[t][e] * rstd;
        dwacc[t][e] += d * xh;
        dv[t][e] = d * wv[t][e];  // g
        xx[t][e] = xh;
        dot += dv[t][e] * xh;
      }
    dot = wave_sum(dot) * invH;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
      const int c = lane + 64 * t;
      if (c < nc) {
        const size_t off = rbase + (size_t)c * 4;
        float dx[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) dx[e] = rstd * (dv[t][e] - xx[t][e] * dot) + rr[t][e];
        st_f4(dx_out + off, dx);
        if (ddelta) {
          u16x4 o;
          if (thr) {
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const uint32_t h = lowbias32(key ^ (uint32_t)((off + e) >> 1));
              o.v[e] = f2h<HK>(((h & 0xffffu) >= thr) ? dx[e] * dscale : 0.f);
              o.v[e + 1] = f2h<HK>(((h >> 16) >= thr) ? dx[e + 1] * dscale : 0.f);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) o.v[e] = f2h<HK>(dx[e]);
          }
          *reinterpret_cast<u16x4*>(ddelta + off) = o;
        }
      }
    }
  }
  // block-reduce dw over the 4 waves -> this block's partial row (dw_part) or, without
  // a workspace, one atomic per column per block
#pragma unroll
  for (int t = 0; t < NCH; ++t) {
    const int c = lane + 64 * t;
    if (c < nc) {
#pragma unroll
      for (int e = 0; e < 4; ++e) smem[wid * H + c * 4 + e] = dwacc[t][e];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < H; j += 256) {
    const float s = smem[j] + smem[H + j] + smem[2 * H + j] + smem[3 * H + j];
    if (dw_part) dw_part[(size_t)blockIdx.x * H + j] = s;
    else unsafeAtomicAdd(dw + j, s);
  }
}

// dw[j] += sum over the partial rows, in a fixed order (bitwise reproducible, no
// float atomics).  One 64*QN-thread block per 4*QN columns: thread (g, q) owns columns
// 4q..4q+3 of the slice (float4 loads, QN threads = one row segment) and rows
// g, g+64, ... with 8 loads in flight (the partials were written by blocks on every XCD,
// so the reads come from the fabric: latency-bound without that parallelism); then the
// 64 row-group sums are added through LDS in two fixed-order levels.
__device__ __forceinline__ void f4add(float4& a, const float4 b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

template <int QN>
__global__ __launch_bounds__(64 * QN) void k_colsum_acc(const float* __restrict__ part, float* __restrict__ dw, int rows,
                                                       int H) {
  constexpr int C = 4 * QN;  // columns per block
  __shared__ float red[64][C + 1];
  __shared__ float red2[16][C];
  const int q = threadIdx.x % QN, g = threadIdx.x / QN;
  const int c0 = blockIdx.x * C + q * 4;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  if (c0 < H) {  // H % 4 == 0: the quad is in range
    const float* p = part + c0;
    int r = g;
    for (; r + 448 < rows; r += 512) {
      float4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = *reinterpret_cast<const float4*>(p + (size_t)(r + 64 * u) * H);
      f4add(a0, x[0]); f4add(a1, x[1]); f4add(a2, x[2]); f4add(a3, x[3]);
      f4add(a0, x[4]); f4add(a1, x[5]); f4add(a2, x[6]); f4add(a3, x[7]);
    }
    for (; r < rows; r += 64) f4add(a0, *reinterpret_cast<const float4*>(p + (size_t)r * H));
  }
  f4add(a0, a1);
  f4add(a2, a3);
  f4add(a0, a2);
  red[g][q * 4 + 0] = a0.x;
  red[g][q * 4 + 1] = a0.y;
  red[g][q * 4 + 2] = a0.z;
  red[g][q * 4 + 3] = a0.w;
  __syncthreads();
  {  // level 2: thread (k, j) adds row groups 4k..4k+3 of column j
    const int j = threadIdx.x % C, k = threadIdx.x / C;
    red2[k][j] = (red[4 * k][j] + red[4 * k + 1][j]) + (red[4 * k + 2][j] + red[4 * k + 3][j]);
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const int j = blockIdx.x * C + threadIdx.x;
    if (j < H) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += red2[k][threadIdx.x];
      dw[j] += s;
    }
  }
}

static inline int nch_of(int H) {
  int n = (H / 4 + 63) / 64;
  if (n > 8 && n <= 12) n = 12;
  else if (n > 12) n = 16;
  return n;
}

// H = 768: the fp32 block input goes out with nontemporal stores (it is read again only
// by the backward, ~10 ms later): step -0.03 / -0.08 / -0.06 ms in three same-box pairs;
// DLT_FWD_NT=0 selects plain stores
static int fwd_nt() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DLT_FWD_NT");
    v = (e && atoi(e) == 0) ? 0 : 1;
  }
  return v;
}

template <int HK>
static void rmsnorm_fwd_launch(int nch, dim3 grid, dim3 block, hipStream_t stream, const float* resid,
                               const bf16_t* delta, const void* w, int wbf16, float* x_out, bf16_t* y_out,
                               float* rstd_out, int M, int H, float eps, uint32_t key, uint32_t thr, float dscale);

// hk: activation format of delta / y_out / a 16-bit weight (0 bf16, 1 fp16)
DLT_API int dlt_add_dropout_rmsnorm_fwd(const float* resid, const bf16_t* delta, const void* w, int wbf16,
                                        float* x_out, bf16_t* y_out, float* rstd_out, int M, int H,
                                        float eps, uint32_t key, uint32_t thr, float dscale, int hk,
                                        hipStream_t stream) {
  if (H % 4 != 0 || H > 4096) return -1;
  const dim3 grid((M + 3) / 4), block(256);
  const int nch = nch_of(H);
  DLT_HK_DISPATCH(hk, rmsnorm_fwd_launch<HKC>(nch, grid, block, stream, resid, delta, w, wbf16, x_out, y_out,
                                              rstd_out, M, H, eps, key, thr, dscale));
  DLT_CHECK_LAUNCH();
}

template <int HK>
static void rmsnorm_fwd_launch(int nch, dim3 grid, dim3 block, hipStream_t stream, const float* resid,
                               const bf16_t* delta, const void* w, int wbf16, float* x_out, bf16_t* y_out,
                               float* rstd_out, int M, int H, float eps, uint32_t key, uint32_t thr, float dscale) {
#define ARGS resid, delta, w, wbf16, x_out, y_out, rstd_out, M, H, eps, key, thr, dscale
  switch (nch) {
    case 1: k_add_dropout_rmsnorm_fwd<1, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 2: k_add_dropout_rmsnorm_fwd<2, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 3:
      if (fwd_nt()) k_add_dropout_rmsnorm_fwd<3, true, HK><<<grid, block, 0, stream>>>(ARGS);
      else k_add_dropout_rmsnorm_fwd<3, false, HK><<<grid, block, 0, stream>>>(ARGS);
      break;
    case 4: k_add_dropout_rmsnorm_fwd<4, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 5: k_add_dropout_rmsnorm_fwd<5, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 6: k_add_dropout_rmsnorm_fwd<6, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 7: k_add_dropout_rmsnorm_fwd<7, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 8: k_add_dropout_rmsnorm_fwd<8, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    case 12: k_add_dropout_rmsnorm_fwd<12, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
    default: k_add_dropout_rmsnorm_fwd<16, false, HK><<<grid, block, 0, stream>>>(ARGS); break;
  }
#undef ARGS
}

template <int HK>
static void rmsnorm_bwd_launch(int nch, dim3 grid, dim3 block, size_t shm, hipStream_t stream, const bf16_t* dy,
                               const float* x, const float* rstd, const void* w, int wbf16, const float* dres,
                               float* dx_out, bf16_t* ddelta, float* dw, float* dw_ws, const float* dy_scale,
                               float dy_mul, int M, int H, uint32_t key, uint32_t thr, float dscale) {
#define ARGS dy, x, rstd, w, wbf16, dres, dx_out, ddelta, dw, dw_ws, dy_scale, dy_mul, M, H, key, thr, dscale
  switch (nch) {
    case 1: k_rmsnorm_bwd<1, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 2: k_rmsnorm_bwd<2, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 3: k_rmsnorm_bwd<3, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 4: k_rmsnorm_bwd<4, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 5: k_rmsnorm_bwd<5, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 6: k_rmsnorm_bwd<6, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 7: k_rmsnorm_bwd<7, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 8: k_rmsnorm_bwd<8, HK><<<grid, block, shm, stream>>>(ARGS); break;
    case 12: k_rmsnorm_bwd<12, HK><<<grid, block, shm, stream>>>(ARGS); break;
    default: k_rmsnorm_bwd<16, HK><<<grid, block, shm, stream>>>(ARGS); break;
  }
#undef ARGS
}

// hk: activation format of dy / ddelta / a 16-bit weight (0 bf16, 1 fp16)
DLT_API int dlt_rmsnorm_bwd(const bf16_t* dy, const float* x, const float* rstd, const void* w, int wbf16,
                            const float* dres, float* dx_out, bf16_t* ddelta, float* dw, float* dw_ws,
                            const float* dy_scale, float dy_mul, int M, int H, uint32_t key, uint32_t thr,
                            float dscale, int hk, hipStream_t stream) {
  if (H % 4 != 0 || H > 4096) return -1;
  // enough waves to cover HBM latency (~2 rows per wave at M = 8192), few enough
  // blocks that the per-block dw atomics stay negligible
  int blocks = (M + 3) / 4;
  if (blocks > 1024) blocks = 1024;
  const dim3 grid(blocks), block(256);
  const size_t shm = (size_t)4 * H * sizeof(float);
  const int nch = nch_of(H);
  DLT_HK_DISPATCH(hk, rmsnorm_bwd_launch<HKC>(nch, grid, block, shm, stream, dy, x, rstd, w, wbf16, dres, dx_out,
                                              ddelta, dw, dw_ws, dy_scale, dy_mul, M, H, key, thr, dscale));
  if (dw_ws) {
    // 16-column blocks of 256 threads (48 for H = 768) slot into the CUs that the other
    // micro-step chain's kernels leave free; 64-column blocks of 1024 threads waited for
    // a whole free CU (45 us in the overlapped step vs 6 us alone).  Same summation order
    // either way (DLT_COLSUM_WIDE=1: the 1024-thread form).
    static const bool wide = getenv("DLT_COLSUM_WIDE") && atoi(getenv("DLT_COLSUM_WIDE")) == 1;
    if (wide) k_colsum_acc<16><<<(H + 63) / 64, 1024, 0, stream>>>(dw_ws, dw, blocks, H);
    else k_colsum_acc<4><<<(H + 15) / 16, 256, 0, stream>>>(dw_ws, dw, blocks, H);
  }
  DLT_CHECK_LAUNCH();
}
