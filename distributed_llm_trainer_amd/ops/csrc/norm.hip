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
// One wave (64 lanes) owns one row; each lane keeps its 8-element chunks in
// registers (MAXC chunks/lane -> H <= MAXC*512), so x is read once.  The residual
// stream is fp32 (matches the reference DDP/autocast numerics).
#include "common.h"

template <int MAXC>
__global__ __launch_bounds__(256) void k_add_dropout_rmsnorm_fwd(
    const float* __restrict__ resid, const bf16_t* __restrict__ delta, const float* __restrict__ w,
    float* __restrict__ x_out, bf16_t* __restrict__ y_out, float* __restrict__ rstd_out,
    int M, int H, float eps, uint32_t key, uint32_t thr, float dscale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nc = H >> 3;
  const size_t rbase = (size_t)row * H;
  float xv[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < nc) {
      const size_t off = rbase + (size_t)c * 8;
      float r[8];
      if (resid) {
        const float4 a = *reinterpret_cast<const float4*>(resid + off);
        const float4 b = *reinterpret_cast<const float4*>(resid + off + 4);
        r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w; r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = 0.f;
      }
      if (delta) {
        const u16x8 d = *reinterpret_cast<const u16x8*>(delta + off);
        if (thr) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const uint32_t h = lowbias32(key ^ (uint32_t)((off + e) >> 1));
            const float d0 = bf2f(d.v[e]), d1 = bf2f(d.v[e + 1]);
            r[e] += ((h & 0xffffu) >= thr) ? d0 * dscale : 0.f;
            r[e + 1] += ((h >> 16) >= thr) ? d1 * dscale : 0.f;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] += bf2f(d.v[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { xv[t][e] = r[e]; ss += r[e] * r[e]; }
    }
  }
  ss = wave_sum(ss);
  const float rstd = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd_out[row] = rstd;
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < nc) {
      const size_t off = rbase + (size_t)c * 8;
      if (x_out) {
        *reinterpret_cast<float4*>(x_out + off) = make_float4(xv[t][0], xv[t][1], xv[t][2], xv[t][3]);
        *reinterpret_cast<float4*>(x_out + off + 4) = make_float4(xv[t][4], xv[t][5], xv[t][6], xv[t][7]);
      }
      const float4 wa = *reinterpret_cast<const float4*>(w + c * 8);
      const float4 wb = *reinterpret_cast<const float4*>(w + c * 8 + 4);
      const float ww[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
      u16x8 y;
#pragma unroll
      for (int e = 0; e < 8; ++e) y.v[e] = f2bf(xv[t][e] * rstd * ww[e]);
      *reinterpret_cast<u16x8*>(y_out + off) = y;
    }
  }
}

template <int MAXC>
__global__ __launch_bounds__(256) void k_rmsnorm_bwd(
    const bf16_t* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ rstd_in,
    const float* __restrict__ w, const float* __restrict__ dres, float* __restrict__ dx_out,
    bf16_t* __restrict__ ddelta, float* __restrict__ dw, const float* __restrict__ dy_scale,
    int M, int H, uint32_t key, uint32_t thr, float dscale) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [4][H]
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nc = H >> 3;
  const float sc = dy_scale ? *dy_scale : 1.f;
  const float invH = 1.f / (float)H;
  float dwacc[MAXC][8];
  float wv[MAXC][8];
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
#pragma unroll
    for (int e = 0; e < 8; ++e) { dwacc[t][e] = 0.f; wv[t][e] = 0.f; }
    if (c < nc) {
      const float4 wa = *reinterpret_cast<const float4*>(w + c * 8);
      const float4 wb = *reinterpret_cast<const float4*>(w + c * 8 + 4);
      wv[t][0] = wa.x; wv[t][1] = wa.y; wv[t][2] = wa.z; wv[t][3] = wa.w;
      wv[t][4] = wb.x; wv[t][5] = wb.y; wv[t][6] = wb.z; wv[t][7] = wb.w;
    }
  }
  for (int row = blockIdx.x * 4 + wid; row < M; row += gridDim.x * 4) {
    const size_t rbase = (size_t)row * H;
    const float rstd = rstd_in[row];
    float g[MAXC][8], xh[MAXC][8];
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < MAXC; ++t) {
      const int c = lane + 64 * t;
      if (c < nc) {
        const size_t off = rbase + (size_t)c * 8;
        const u16x8 d = *reinterpret_cast<const u16x8*>(dy + off);
        const float4 a = *reinterpret_cast<const float4*>(x + off);
        const float4 b = *reinterpret_cast<const float4*>(x + off + 4);
        const float xx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dv = bf2f(d.v[e]) * sc;
          xh[t][e] = xx[e] * rstd;
          dwacc[t][e] += dv * xh[t][e];
          g[t][e] = dv * wv[t][e];
          dot += g[t][e] * xh[t][e];
        }
      }
    }
    dot = wave_sum(dot) * invH;
#pragma unroll
    for (int t = 0; t < MAXC; ++t) {
      const int c = lane + 64 * t;
      if (c < nc) {
        const size_t off = rbase + (size_t)c * 8;
        float dx[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) dx[e] = rstd * (g[t][e] - xh[t][e] * dot);
        if (dres) {
          const float4 a = *reinterpret_cast<const float4*>(dres + off);
          const float4 b = *reinterpret_cast<const float4*>(dres + off + 4);
          dx[0] += a.x; dx[1] += a.y; dx[2] += a.z; dx[3] += a.w;
          dx[4] += b.x; dx[5] += b.y; dx[6] += b.z; dx[7] += b.w;
        }
        *reinterpret_cast<float4*>(dx_out + off) = make_float4(dx[0], dx[1], dx[2], dx[3]);
        *reinterpret_cast<float4*>(dx_out + off + 4) = make_float4(dx[4], dx[5], dx[6], dx[7]);
        if (ddelta) {
          u16x8 o;
          if (thr) {
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const uint32_t h = lowbias32(key ^ (uint32_t)((off + e) >> 1));
              o.v[e] = f2bf(((h & 0xffffu) >= thr) ? dx[e] * dscale : 0.f);
              o.v[e + 1] = f2bf(((h >> 16) >= thr) ? dx[e + 1] * dscale : 0.f);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o.v[e] = f2bf(dx[e]);
          }
          *reinterpret_cast<u16x8*>(ddelta + off) = o;
        }
      }
    }
  }
  // block-reduce dw over the 4 waves, then one atomic per column per block
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < nc) {
#pragma unroll
      for (int e = 0; e < 8; ++e) smem[wid * H + c * 8 + e] = dwacc[t][e];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < H; j += 256) {
    const float s = smem[j] + smem[H + j] + smem[2 * H + j] + smem[3 * H + j];
    unsafeAtomicAdd(dw + j, s);
  }
}

DLT_API int dlt_add_dropout_rmsnorm_fwd(const float* resid, const bf16_t* delta, const float* w,
                                        float* x_out, bf16_t* y_out, float* rstd_out, int M, int H,
                                        float eps, uint32_t key, uint32_t thr, float dscale,
                                        hipStream_t stream) {
  if (H % 8 != 0 || H > 4096) return -1;
  const dim3 grid((M + 3) / 4), block(256);
  const int nc = H / 8;
  if (nc <= 64)
    k_add_dropout_rmsnorm_fwd<1><<<grid, block, 0, stream>>>(resid, delta, w, x_out, y_out, rstd_out, M, H, eps, key, thr, dscale);
  else if (nc <= 128)
    k_add_dropout_rmsnorm_fwd<2><<<grid, block, 0, stream>>>(resid, delta, w, x_out, y_out, rstd_out, M, H, eps, key, thr, dscale);
  else if (nc <= 256)
    k_add_dropout_rmsnorm_fwd<4><<<grid, block, 0, stream>>>(resid, delta, w, x_out, y_out, rstd_out, M, H, eps, key, thr, dscale);
  else
    k_add_dropout_rmsnorm_fwd<8><<<grid, block, 0, stream>>>(resid, delta, w, x_out, y_out, rstd_out, M, H, eps, key, thr, dscale);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_rmsnorm_bwd(const bf16_t* dy, const float* x, const float* rstd, const float* w,
                            const float* dres, float* dx_out, bf16_t* ddelta, float* dw,
                            const float* dy_scale, int M, int H, uint32_t key, uint32_t thr,
                            float dscale, hipStream_t stream) {
  if (H % 8 != 0 || H > 4096) return -1;
  int blocks = (M + 3) / 4;
  if (blocks > 1024) blocks = 1024;
  const dim3 grid(blocks), block(256);
  const size_t shm = (size_t)4 * H * sizeof(float);
  const int nc = H / 8;
  if (nc <= 64)
    k_rmsnorm_bwd<1><<<grid, block, shm, stream>>>(dy, x, rstd, w, dres, dx_out, ddelta, dw, dy_scale, M, H, key, thr, dscale);
  else if (nc <= 128)
    k_rmsnorm_bwd<2><<<grid, block, shm, stream>>>(dy, x, rstd, w, dres, dx_out, ddelta, dw, dy_scale, M, H, key, thr, dscale);
  else if (nc <= 256)
    k_rmsnorm_bwd<4><<<grid, block, shm, stream>>>(dy, x, rstd, w, dres, dx_out, ddelta, dw, dy_scale, M, H, key, thr, dscale);
  else
    k_rmsnorm_bwd<8><<<grid, block, shm, stream>>>(dy, x, rstd, w, dres, dx_out, ddelta, dw, dy_scale, M, H, key, thr, dscale);
  DLT_CHECK_LAUNCH();
}
