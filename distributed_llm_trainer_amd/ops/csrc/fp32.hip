// fp32-activation kernels: the engine's `--mixed_precision fp32` mode (the reference's
// fp32 path, ddp_trainer.py:137-139, and FSDP without MixedPrecision, fsdp_trainer.py:223-234)
// on HIP kernels instead of PyTorch ops.  Same contracts and the same dropout bits as the
// 16-bit kernels (ops/reference.py defines both):
//
//   * k_f32_norm_fwd / k_f32_norm_bwd  -- residual add + dropout + RMSNorm and its backward
//     (fp32 y / dy / ddelta; deterministic per-block column partials for dw)
//   * k_f32_rope                       -- NeoX rotation of q / k between any two strided
//     q|k|v layouts (packed [B*S, 3H] <-> head-major [B, nh, S, hd]), forward or inverse
//   * k_f32_swiglu_fwd / _bwd, k_f32_ce_row, k_f32_scale
//   * k_f32_attn_fwd / _bwd_dq / _bwd_dkdv -- causal flash attention, one lane per query
//     (forward, dQ) or per key (dK/dV), K/V (Q/dO) tiles staged through LDS and read as
//     wave-wide broadcasts; head_dim 64 and 128; dropout from the keep-bit words of
//     k_dropout_bits (attention.hip), so fp32 and 16-bit runs drop the same scores.
//     (the default fp32 attention up to 4096 keys is the GEMM formulation instead: its row
//     kernels are in attn_gemm.hip)
//
// fp32 is the reference / debug precision here: these kernels are written for exactness
// and simplicity, not tuned like the bf16 hot path.
#include "common.h"

#include <cfloat>

namespace {

__device__ __forceinline__ bool f32_keep(uint32_t key, uint64_t idx, uint32_t thr) {
  return !thr || drop_bits(key, idx) >= thr;
}

}  // namespace

// ------------------------------------------------------------------ RMSNorm
// One wave per row, lane l owns columns 4l + 256t (t < NT).
template <int NT>
__global__ __launch_bounds__(256) void k_f32_norm_fwd(const float* __restrict__ resid, const float* __restrict__ delta,
                                                      const float* __restrict__ w, float* __restrict__ x_out,
                                                      float* __restrict__ y, float* __restrict__ rstd_out, int M, int H,
                                                      float eps, uint32_t key, uint32_t thr, float dscale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const size_t rb = (size_t)row * H;
  float xv[NT][4];
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = 4 * lane + 256 * t;
#pragma unroll
    for (int e = 0; e < 4; ++e) xv[t][e] = 0.f;
    if (c < H) {
      float4 r = resid ? *reinterpret_cast<const float4*>(resid + rb + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      float rv[4] = {r.x, r.y, r.z, r.w};
      if (delta) {
        const float4 d = *reinterpret_cast<const float4*>(delta + rb + c);
        const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) rv[e] += f32_keep(key, rb + c + e, thr) ? dv[e] * dscale : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xv[t][e] = rv[e];
        ss += rv[e] * rv[e];
      }
      if (x_out) *reinterpret_cast<float4*>(x_out + rb + c) = make_float4(rv[0], rv[1], rv[2], rv[3]);
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd_out[row] = rs;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = 4 * lane + 256 * t;
    if (c < H) {
      const float4 wv = *reinterpret_cast<const float4*>(w + c);
      *reinterpret_cast<float4*>(y + rb + c) =
          make_float4(xv[t][0] * rs * wv.x, xv[t][1] * rs * wv.y, xv[t][2] * rs * wv.z, xv[t][3] * rs * wv.w);
    }
  }
}

// dx = dres + rstd (g - xh mean(g xh)), g = dy * w * scale;  ddelta = keep(dx) / (1 - p);
// dw partial of this block (its 4 waves' rows, fixed order) -> ws[block][H]
template <int NT>
__global__ __launch_bounds__(256) void k_f32_norm_bwd(const float* __restrict__ dy, const float* __restrict__ x,
                                                      const float* __restrict__ rstd, const float* __restrict__ w,
                                                      const float* __restrict__ dres, float* __restrict__ dx_out,
                                                      float* __restrict__ ddelta, float* __restrict__ ws,
                                                      const float* __restrict__ scale_ptr, float dy_mul, int M, int H,
                                                      int rows_per_block, uint32_t key, uint32_t thr, float dscale) {
  __shared__ float red[4][NT * 256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float sc = (scale_ptr ? scale_ptr[0] : 1.f) * dy_mul;
  float dwp[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) dwp[t][e] = 0.f;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int row = r0 + wv; row < r1; row += 4) {
    const size_t rb = (size_t)row * H;
    const float rs = rstd[row];
    float g[NT][4], xh[NT][4];
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = 4 * lane + 256 * t;
#pragma unroll
      for (int e = 0; e < 4; ++e) g[t][e] = xh[t][e] = 0.f;
      if (c < H) {
        const float4 d = *reinterpret_cast<const float4*>(dy + rb + c);
        const float4 xx = *reinterpret_cast<const float4*>(x + rb + c);
        const float4 ww = *reinterpret_cast<const float4*>(w + c);
        const float dv[4] = {d.x * sc, d.y * sc, d.z * sc, d.w * sc};
        const float xv[4] = {xx.x, xx.y, xx.z, xx.w}, wvv[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[t][e] = xv[e] * rs;
          g[t][e] = dv[e] * wvv[e];
          dwp[t][e] += dv[e] * xh[t][e];
          dot += g[t][e] * xh[t][e];
        }
      }
    }
    dot = wave_sum(dot) / (float)H;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = 4 * lane + 256 * t;
      if (c < H) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (g[t][e] - xh[t][e] * dot);
        if (dres) {
          const float4 r = *reinterpret_cast<const float4*>(dres + rb + c);
          o[0] += r.x;
          o[1] += r.y;
          o[2] += r.z;
          o[3] += r.w;
        }
        *reinterpret_cast<float4*>(dx_out + rb + c) = make_float4(o[0], o[1], o[2], o[3]);
        if (ddelta) {
          float dd[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) dd[e] = f32_keep(key, rb + c + e, thr) ? o[e] * dscale : 0.f;
          *reinterpret_cast<float4*>(ddelta + rb + c) = make_float4(dd[0], dd[1], dd[2], dd[3]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wv][256 * t + 4 * lane + e] = dwp[t][e];
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256)
    ws[(size_t)blockIdx.x * H + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// dw[c] += sum_b ws[b][c] in a fixed order (deterministic): 64 columns per workgroup, lane =
// column; wave w of 16 sums rows w, w+16, ... into 4 interleaved accumulators (four loads in
// flight per lane), then the 16 wave sums combine in LDS in wave order.
__global__ __launch_bounds__(1024) void k_f32_colsum(const float* __restrict__ ws, float* __restrict__ dw, int nb, int H) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < H) {
    int b = w;
    for (; b + 48 < nb; b += 64) {
      a0 += ws[(size_t)b * H + c];
      a1 += ws[(size_t)(b + 16) * H + c];
      a2 += ws[(size_t)(b + 32) * H + c];
      a3 += ws[(size_t)(b + 48) * H + c];
    }
    for (; b < nb; b += 16) a0 += ws[(size_t)b * H + c];
  }
  part[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && c < H) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += part[i][lane];
    dw[c] += s;
  }
}

// ------------------------------------------------------------------- RoPE
// For tensor t in {q, k, v} (t < 2 rotated, sign -1 = inverse rotation), element (b, s, h, j):
//   src at src_t + b*sb + s*sr + h*sh + j, dst likewise with the d* strides.
// In place is allowed (same pointer and strides).  Grid x: (head, pair j) of a row, one
// thread each; grid y strides over the B*S rows (no 64-bit index division per element).
// cosT == nullptr: a plain layout copy of the ntens tensors (no rotation).
struct F32QKV {
  const float* src[3];
  float* dst[3];
  long sb, sr, sh, db, dr, dh;
};

__global__ __launch_bounds__(256) void k_f32_rope(F32QKV a, const float* __restrict__ cosT,
                                                  const float* __restrict__ sinT, int B, int S, int nh, int hd,
                                                  float sign, int ntens) {
  const int half = hd >> 1;
  const int t0 = blockIdx.x * 256 + threadIdx.x;
  if (t0 >= nh * half) return;
  const int h = t0 / half, j = t0 - h * half;
  for (int r = blockIdx.y; r < B * S; r += gridDim.y) {
    const int b = r / S, s = r - b * S;
    const bool rot = cosT != nullptr;
    const float c = rot ? cosT[(size_t)s * half + j] : 1.f, sn = rot ? sign * sinT[(size_t)s * half + j] : 0.f;
    const long so = b * a.sb + s * a.sr + h * a.sh + j, dof = b * a.db + s * a.dr + h * a.dh + j;
    for (int t = 0; t < ntens; ++t) {
      const float x1 = a.src[t][so], x2 = a.src[t][so + half];
      if (t < 2 && rot) {
        a.dst[t][dof] = x1 * c - x2 * sn;
        a.dst[t][dof + half] = x2 * c + x1 * sn;
      } else {
        a.dst[t][dof] = x1;
        a.dst[t][dof + half] = x2;
      }
    }
  }
}

// The copy mode of k_f32_rope with float4 accesses: 4 consecutive elements of a head row per
// thread (hd % 4 == 0, every stride a multiple of 4 elements, 16-byte aligned bases).
__global__ __launch_bounds__(256) void k_f32_relayout4(F32QKV a, int B, int S, int nh, int hd, int ntens) {
  const int per = hd >> 2;
  const int t0 = blockIdx.x * 256 + threadIdx.x;
  if (t0 >= nh * per) return;
  const int h = t0 / per, j = (t0 - h * per) * 4;
  for (int r = blockIdx.y; r < B * S; r += gridDim.y) {
    const int b = r / S, s = r - b * S;
    const long so = b * a.sb + s * a.sr + h * a.sh + j, dof = b * a.db + s * a.dr + h * a.dh + j;
    for (int t = 0; t < ntens; ++t)
      *reinterpret_cast<float4*>(a.dst[t] + dof) = *reinterpret_cast<const float4*>(a.src[t] + so);
  }
}

// ----------------------------------------------------------------- SwiGLU
// Grid x: V consecutive columns per thread (V = 4: float4 accesses, I % 4 == 0); grid y
// strides over the rows.
template <int V>
struct F32Vec {
  float v[V];
};

template <int V>
__device__ __forceinline__ F32Vec<V> f32_ldv(const float* p) {
  F32Vec<V> r;
  if constexpr (V == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) r.v[i] = p[i];
  }
  return r;
}

template <int V>
__device__ __forceinline__ void f32_stv(float* p, const F32Vec<V>& r) {
  if constexpr (V == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i] = r.v[i];
  }
}

template <int V>
__global__ __launch_bounds__(256) void k_f32_swiglu_fwd(const float* __restrict__ gu, float* __restrict__ s, int M, int I) {
  const int j = (blockIdx.x * 256 + threadIdx.x) * V;
  if (j >= I) return;
  for (int m = blockIdx.y; m < M; m += gridDim.y) {
    const float* row = gu + (size_t)m * 2 * I;
    const F32Vec<V> g = f32_ldv<V>(row + j), u = f32_ldv<V>(row + I + j);
    F32Vec<V> o;
#pragma unroll
    for (int i = 0; i < V; ++i) o.v[i] = g.v[i] * dlt_sigmoid(g.v[i]) * u.v[i];
    f32_stv<V>(s + (size_t)m * I + j, o);
  }
}

template <int V>
__global__ __launch_bounds__(256) void k_f32_swiglu_bwd(const float* __restrict__ gu, const float* __restrict__ da,
                                                        float* __restrict__ dgu, float* __restrict__ s_out, int M,
                                                        int I) {
  const int j = (blockIdx.x * 256 + threadIdx.x) * V;
  if (j >= I) return;
  for (int m = blockIdx.y; m < M; m += gridDim.y) {
    const float* row = gu + (size_t)m * 2 * I;
    const F32Vec<V> g = f32_ldv<V>(row + j), u = f32_ldv<V>(row + I + j), d = f32_ldv<V>(da + (size_t)m * I + j);
    F32Vec<V> dg, du, so;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const float sg = dlt_sigmoid(g.v[i]);
      dg.v[i] = d.v[i] * u.v[i] * sg * (1.f + g.v[i] * (1.f - sg));
      du.v[i] = d.v[i] * g.v[i] * sg;
      so.v[i] = g.v[i] * sg * u.v[i];
    }
    float* drow = dgu + (size_t)m * 2 * I;
    f32_stv<V>(drow + j, dg);
    f32_stv<V>(drow + I + j, du);
    if (s_out) f32_stv<V>(s_out + (size_t)m * I + j, so);
  }
}

// ----------------------------------------------------------- cross-entropy
// One 256-thread block per row: logsumexp over the first `vocab` columns (online max /
// sum per thread, then block combine), loss = lse - logit[target], and the row is
// overwritten by grad_scale * (softmax - onehot) / n_valid (padding columns and ignored
// rows: zero).
template <int V>
__global__ __launch_bounds__(256) void k_f32_ce_row(float* __restrict__ logits, const long* __restrict__ targets,
                                                    const long* __restrict__ n_valid, float* __restrict__ loss, int Vp,
                                                    int vocab, float grad_scale) {
  __shared__ float sm[4], sl[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  float* lg = logits + (size_t)row * Vp;
  const long tg = targets[row];
  float m = -INFINITY, l = 0.f;
  // V-wide groups (one rescale per group), then the scalar tail of vocab % V columns
  const int nvg = vocab / V;
  for (int c = tid; c < nvg; c += 256) {
    const F32Vec<V> x = f32_ldv<V>(lg + c * V);
    float mx = x.v[0];
#pragma unroll
    for (int i = 1; i < V; ++i) mx = fmaxf(mx, x.v[i]);
    if (mx > m) {
      l *= __expf(m - mx);
      m = mx;
    }
#pragma unroll
    for (int i = 0; i < V; ++i) l += __expf(x.v[i] - m);
  }
  for (int c = nvg * V + tid; c < vocab; c += 256) {
    const float v = lg[c];
    if (v > m) {
      l = l * __expf(m - v) + 1.f;
      m = v;
    } else {
      l += __expf(v - m);
    }
  }
  // block combine: wave then across the 4 waves
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
    const float mm = fmaxf(m, m2);
    l = (m == -INFINITY ? 0.f : l * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - mm));
    m = mm;
  }
  if ((tid & 63) == 0) {
    sm[tid >> 6] = m;
    sl[tid >> 6] = l;
  }
  __syncthreads();
  float M4 = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  float L4 = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) L4 += sm[k] == -INFINITY ? 0.f : sl[k] * __expf(sm[k] - M4);
  const float lse = M4 + __logf(L4);
  const bool valid = tg != -100;
  const float nv = (float)(n_valid[0] > 0 ? n_valid[0] : 1);
  if (tid == 0) loss[row] = valid ? lse - lg[tg] : 0.f;
  __syncthreads();  // the target logit is read before any thread overwrites it
  const float gs = valid ? grad_scale / nv : 0.f;
  for (int c0 = tid * V; c0 < Vp; c0 += 256 * V) {
    F32Vec<V> g = f32_ldv<V>(lg + c0);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = c0 + i;
      g.v[i] = (c < vocab && valid) ? (__expf(g.v[i] - lse) - (c == tg ? 1.f : 0.f)) * gs : 0.f;
    }
    f32_stv<V>(lg + c0, g);
  }
}

__global__ __launch_bounds__(256) void k_f32_scale(const float* __restrict__ x, float* __restrict__ y, long n,
                                                   const float* __restrict__ s, float mul) {
  const float f = s[0] * mul;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = x[i] * f;
}

// -------------------------------------------------------------- attention
// q / k / v / dq / dk / dv: element (b, h, s, d) at base + b*bs + h*hs + s*rs + d;
// o / do: [B*S, nh*HD]; lse / delta: [B*nh, S] (natural log); mask: [2, B*nh, W, S] keep
// words (attention.hip k_dropout_bits: [0] row layout word (bh, w, q) bit j = keep(q, 32w+j),
// [1] transposed word (bh, w, k) bit j = keep(32w+j, k)).
struct F32Attn {
  const float* q;
  const float* k;
  const float* v;
  long bs, hs, rs;  // q / k / v strides
  float* dq;
  float* dk;
  float* dv;
  long gbs, ghs, grs;  // dq / dk / dv strides
  const float* o;
  const float* dO;
  float* out;   // forward output o
  float* lse;   // forward: written; backward: read
  float* delta; // backward: rowsum(dO * O), written by the dQ kernel
  const uint32_t* mask;
  int B, nh, S;
  float scale, dscale;
};

constexpr int F32_T = 64;  // keys (queries) per LDS tile; one wave per workgroup

template <int HD>
__global__ __launch_bounds__(64) void k_f32_attn_fwd(F32Attn a) {
  __shared__ float Ks[F32_T][HD], Vs[F32_T][HD];
  __shared__ float Ss[F32_T][64];  // the lane's scores of the tile (a private LDS column)
  const int lane = threadIdx.x;
  const int bh = blockIdx.y, b = bh / a.nh, h = bh % a.nh;
  const int qi = blockIdx.x * F32_T + lane;
  const int S = a.S, W = (S + 31) >> 5;
  const long base = (long)b * a.bs + (long)h * a.hs;
  const float cl2 = a.scale * 1.44269504088896341f;
  float qv[HD], ov[HD];
  const int qc = min(qi, S - 1);
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    qv[d] = a.q[base + (long)qc * a.rs + d] * cl2;
    ov[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const uint32_t* mrow = a.mask ? a.mask + (size_t)bh * W * S + qc : nullptr;
  const int nkt = min(blockIdx.x + 1, (S + F32_T - 1) / F32_T);
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * F32_T;
    __syncthreads();
    for (int e = lane; e < F32_T * HD; e += 64) {
      const int r = e / HD, d = e - r * HD, kr = min(k0 + r, S - 1);
      Ks[r][d] = a.k[base + (long)kr * a.rs + d];
      Vs[r][d] = a.v[base + (long)kr * a.rs + d];
    }
    __syncthreads();
    float mx = -INFINITY;
    for (int j = 0; j < F32_T; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) acc = fmaf(qv[d], Ks[j][d], acc);
      const int kj = k0 + j;
      const float sj = (kj > qi || kj >= S) ? -INFINITY : acc;
      Ss[j][lane] = sj;
      mx = fmaxf(mx, sj);
    }
    const float mn = fmaxf(m, mx);
    if (mn == -INFINITY) continue;  // a query past S (masked row): nothing to add
    const float corr = exp2f(m - mn);
    l *= corr;
#pragma unroll
    for (int d = 0; d < HD; ++d) ov[d] *= corr;
    m = mn;
    const uint32_t w0 = mrow ? mrow[(size_t)(2 * kt) * S] : ~0u;
    const uint32_t w1 = (mrow && 2 * kt + 1 < W) ? mrow[(size_t)(2 * kt + 1) * S] : ~0u;
    for (int j = 0; j < F32_T; ++j) {
      const float p = exp2f(Ss[j][lane] - m);
      l += p;
      const bool keep = ((j < 32 ? w0 : w1) >> (j & 31)) & 1u;
      const float pd = mrow ? (keep ? p * a.dscale : 0.f) : p;
      if (pd != 0.f) {
#pragma unroll
        for (int d = 0; d < HD; ++d) ov[d] = fmaf(pd, Vs[j][d], ov[d]);
      }
    }
  }
  if (qi < S) {
    const float inv = 1.f / l;
    float* orow = a.out + ((size_t)b * S + qi) * (size_t)(a.nh * HD) + (size_t)h * HD;
#pragma unroll
    for (int d = 0; d < HD; ++d) orow[d] = ov[d] * inv;
    a.lse[(size_t)bh * S + qi] = (m + __log2f(l)) * 0.69314718055994531f;
  }
}

// dQ (and delta = rowsum(dO * O)): one lane per query, K / V tiles through LDS
// HD 128: the dQ accumulator lives in a lane-private LDS column (registers: q, dO).
template <int HD>
__global__ __launch_bounds__(64) void k_f32_attn_bwd_dq(F32Attn a) {
  constexpr bool ACC_LDS = HD > 64;
  __shared__ float Ks[F32_T][HD], Vs[F32_T][HD];
  __shared__ float dqs[ACC_LDS ? HD : 1][64];
  const int lane = threadIdx.x;
  const int bh = blockIdx.y, b = bh / a.nh, h = bh % a.nh;
  const int qi = blockIdx.x * F32_T + lane;
  const int S = a.S, W = (S + 31) >> 5;
  const long base = (long)b * a.bs + (long)h * a.hs;
  const int qc = min(qi, S - 1);
  const float* dorow = a.dO + ((size_t)b * S + qc) * (size_t)(a.nh * HD) + (size_t)h * HD;
  const float* orow = a.o + ((size_t)b * S + qc) * (size_t)(a.nh * HD) + (size_t)h * HD;
  float qv[HD], dov[HD], dqv[ACC_LDS ? 1 : HD];
  float delta = 0.f;
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    qv[d] = a.q[base + (long)qc * a.rs + d];
    dov[d] = dorow[d];
    delta = fmaf(dov[d], orow[d], delta);
    if constexpr (ACC_LDS) dqs[d][lane] = 0.f;
    else dqv[d] = 0.f;
  }
  if (qi < S) a.delta[(size_t)bh * S + qi] = delta;
  const float lse = a.lse[(size_t)bh * S + qc];
  const uint32_t* mrow = a.mask ? a.mask + (size_t)bh * W * S + qc : nullptr;
  const int nkt = min(blockIdx.x + 1, (S + F32_T - 1) / F32_T);
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * F32_T;
    __syncthreads();
    for (int e = lane; e < F32_T * HD; e += 64) {
      const int r = e / HD, d = e - r * HD, kr = min(k0 + r, S - 1);
      Ks[r][d] = a.k[base + (long)kr * a.rs + d];
      Vs[r][d] = a.v[base + (long)kr * a.rs + d];
    }
    __syncthreads();
    const uint32_t w0 = mrow ? mrow[(size_t)(2 * kt) * S] : ~0u;
    const uint32_t w1 = (mrow && 2 * kt + 1 < W) ? mrow[(size_t)(2 * kt + 1) * S] : ~0u;
    for (int j = 0; j < F32_T; ++j) {
      const int kj = k0 + j;
      if (kj > qi || kj >= S) break;  // causal: keys beyond the query end the tile
      float sacc = 0.f, dpv = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) {
        sacc = fmaf(qv[d], Ks[j][d], sacc);
        dpv = fmaf(dov[d], Vs[j][d], dpv);
      }
      const float p = __expf(sacc * a.scale - lse);
      const bool keep = ((j < 32 ? w0 : w1) >> (j & 31)) & 1u;
      const float dp = mrow ? (keep ? dpv * a.dscale : 0.f) : dpv;
      const float ds = p * (dp - delta) * a.scale;
#pragma unroll
      for (int d = 0; d < HD; ++d) {
        if constexpr (ACC_LDS) dqs[d][lane] = fmaf(ds, Ks[j][d], dqs[d][lane]);
        else dqv[d] = fmaf(ds, Ks[j][d], dqv[d]);
      }
    }
  }
  if (qi < S) {
    float* g = a.dq + (long)b * a.gbs + (long)h * a.ghs + (long)qi * a.grs;
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      if constexpr (ACC_LDS) g[d] = dqs[d][lane];
      else g[d] = dqv[d];
    }
  }
}

// dK / dV: one lane per key, Q / dO tiles (plus their lse / delta) through LDS.
// HD 128: the dK / dV accumulators and the key's v row live in lane-private LDS columns
// (registers: k) and the Q / dO tiles are 32 rows, so the workgroup fits in LDS.
template <int HD>
__global__ __launch_bounds__(64) void k_f32_attn_bwd_dkdv(F32Attn a) {
  constexpr bool BIG = HD > 64;
  constexpr int TQ = BIG ? 32 : F32_T;  // queries per LDS tile
  __shared__ float Qs[TQ][HD], Ds[TQ][HD], Ls[TQ], Es[TQ];
  __shared__ float dvs[BIG ? HD : 1][64], dks[BIG ? HD : 1][64], vvs[BIG ? HD : 1][64];
  const int lane = threadIdx.x;
  const int bh = blockIdx.y, b = bh / a.nh, h = bh % a.nh;
  const int ki = blockIdx.x * F32_T + lane;
  const int S = a.S, W = (S + 31) >> 5;
  const long base = (long)b * a.bs + (long)h * a.hs;
  const int kc = min(ki, S - 1);
  float kv[HD], vv[BIG ? 1 : HD], dkv[BIG ? 1 : HD], dvr[BIG ? 1 : HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    kv[d] = a.k[base + (long)kc * a.rs + d];
    const float vd = a.v[base + (long)kc * a.rs + d];
    if constexpr (BIG) {
      vvs[d][lane] = vd;
      dvs[d][lane] = 0.f;
      dks[d][lane] = 0.f;
    } else {
      vv[d] = vd;
      dvr[d] = 0.f;
      dkv[d] = 0.f;
    }
  }
  const uint32_t* mT = a.mask ? a.mask + (size_t)a.B * a.nh * W * S + (size_t)bh * W * S + kc : nullptr;
  const int nqt = (S + TQ - 1) / TQ;
  for (int qt = blockIdx.x * (F32_T / TQ); qt < nqt; ++qt) {
    const int q0 = qt * TQ;
    __syncthreads();
    for (int e = lane; e < TQ * HD; e += 64) {
      const int r = e / HD, d = e - r * HD, qr = min(q0 + r, S - 1);
      Qs[r][d] = a.q[base + (long)qr * a.rs + d];
      Ds[r][d] = a.dO[((size_t)b * S + qr) * (size_t)(a.nh * HD) + (size_t)h * HD + d];
    }
    if (lane < TQ) {
      const int qr = min(q0 + lane, S - 1);
      Ls[lane] = a.lse[(size_t)bh * S + qr];
      Es[lane] = a.delta[(size_t)bh * S + qr];
    }
    __syncthreads();
    const int wq = q0 >> 5;
    const uint32_t w0 = mT ? mT[(size_t)wq * S] : ~0u;
    const uint32_t w1 = (TQ > 32 && mT && wq + 1 < W) ? mT[(size_t)(wq + 1) * S] : ~0u;
    for (int i = 0; i < TQ; ++i) {
      const int qi = q0 + i;
      if (qi >= S) break;
      if (qi < ki) continue;  // causal: only queries at or after this key
      float sacc = 0.f, dpv = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) {
        sacc = fmaf(kv[d], Qs[i][d], sacc);
        if constexpr (BIG) dpv = fmaf(vvs[d][lane], Ds[i][d], dpv);
        else dpv = fmaf(vv[d], Ds[i][d], dpv);
      }
      const float p = __expf(sacc * a.scale - Ls[i]);
      const bool keep = ((i < 32 ? w0 : w1) >> (i & 31)) & 1u;
      const float pd = mT ? (keep ? p * a.dscale : 0.f) : p;
      const float dp = mT ? (keep ? dpv * a.dscale : 0.f) : dpv;
      const float ds = p * (dp - Es[i]) * a.scale;
#pragma unroll
      for (int d = 0; d < HD; ++d) {
        if constexpr (BIG) {
          dks[d][lane] = fmaf(ds, Qs[i][d], dks[d][lane]);
          dvs[d][lane] = fmaf(pd, Ds[i][d], dvs[d][lane]);
        } else {
          dkv[d] = fmaf(ds, Qs[i][d], dkv[d]);
          dvr[d] = fmaf(pd, Ds[i][d], dvr[d]);
        }
      }
    }
  }
  if (ki < S) {
    float* gk = a.dk + (long)b * a.gbs + (long)h * a.ghs + (long)ki * a.grs;
    float* gv = a.dv + (long)b * a.gbs + (long)h * a.ghs + (long)ki * a.grs;
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      if constexpr (BIG) {
        gk[d] = dks[d][lane];
        gv[d] = dvs[d][lane];
      } else {
        gk[d] = dkv[d];
        gv[d] = dvr[d];
      }
    }
  }
}

// ---------------------------------------------------------------- launchers
static inline int f32_blocks(long n) {
  long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

#define F32_NT_DISPATCH(nt, ...)                                   \
  switch (nt) {                                                    \
    case 1: { constexpr int NTC = 1; __VA_ARGS__; } break;         \
    case 2: { constexpr int NTC = 2; __VA_ARGS__; } break;         \
    case 3: { constexpr int NTC = 3; __VA_ARGS__; } break;         \
    case 4: { constexpr int NTC = 4; __VA_ARGS__; } break;         \
    case 5: { constexpr int NTC = 5; __VA_ARGS__; } break;         \
    case 6: { constexpr int NTC = 6; __VA_ARGS__; } break;         \
    case 7: { constexpr int NTC = 7; __VA_ARGS__; } break;         \
    case 8: { constexpr int NTC = 8; __VA_ARGS__; } break;         \
    default: return -1;                                            \
  }

DLT_API int dlt_f32_norm_fwd(const float* resid, const float* delta, const float* w, float* x_out, float* y, float* rstd,
                             int M, int H, float eps, uint32_t key, uint32_t thr, float dscale, hipStream_t st) {
  if (H % 4 || H > 2048) return -1;
  const int nt = (H + 255) / 256;
  F32_NT_DISPATCH(nt, k_f32_norm_fwd<NTC><<<(M + 3) / 4, 256, 0, st>>>(resid, delta, w, x_out, y, rstd, M, H, eps, key,
                                                                       thr, dscale));
  DLT_CHECK_LAUNCH();
}

// ws: nb * H floats with nb = min(1024, ceil(M / 4)); returns -1 for H % 4 or H > 2048
DLT_API int dlt_f32_norm_bwd(const float* dy, const float* x, const float* rstd, const float* w, const float* dres,
                             float* dx, float* ddelta, float* dweight, float* ws, const float* scale, float dy_mul, int M,
                             int H, uint32_t key, uint32_t thr, float dscale, hipStream_t st) {
  if (H % 4 || H > 2048 || M <= 0) return -1;
  const int nt = (H + 255) / 256;
  int nb = (M + 3) / 4;
  if (nb > 1024) nb = 1024;
  const int rpb = (M + nb - 1) / nb;
  nb = (M + rpb - 1) / rpb;
  F32_NT_DISPATCH(nt, k_f32_norm_bwd<NTC><<<nb, 256, 0, st>>>(dy, x, rstd, w, dres, dx, ddelta, ws, scale, dy_mul, M, H,
                                                              rpb, key, thr, dscale));
  k_f32_colsum<<<(H + 63) / 64, 1024, 0, st>>>(ws, dweight, nb, H);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_f32_rope(const float* sq, const float* sk, const float* sv, float* dq, float* dk, float* dv, long sb,
                         long sr, long sh, long db, long dr, long dh, const float* cosT, const float* sinT, int B, int S,
                         int nh, int hd, float sign, int ntens, hipStream_t st) {
  if (hd % 2 || ntens < 1 || ntens > 3 || (cosT && ntens < 2)) return -1;
  F32QKV a{{sq, sk, sv}, {dq, dk, dv}, sb, sr, sh, db, dr, dh};
  if ((long)B * S > 0x7fffffffL) return -1;
  if (!cosT) {  // plain layout copy: float4 when every address lines up
    bool v4 = hd % 4 == 0;
    for (long x : {sb, sr, sh, db, dr, dh}) v4 = v4 && x % 4 == 0;
    for (int t = 0; t < ntens; ++t) v4 = v4 && ((uintptr_t)a.src[t] & 15) == 0 && ((uintptr_t)a.dst[t] & 15) == 0;
    if (v4) {
      const dim3 g4((nh * (hd / 4) + 255) / 256, B * S < 65535 ? B * S : 65535);
      k_f32_relayout4<<<g4, 256, 0, st>>>(a, B, S, nh, hd, ntens);
      DLT_CHECK_LAUNCH();
    }
  }
  const dim3 grid((nh * (hd / 2) + 255) / 256, B * S < 65535 ? B * S : 65535);
  k_f32_rope<<<grid, 256, 0, st>>>(a, cosT, sinT, B, S, nh, hd, sign, ntens);
  DLT_CHECK_LAUNCH();
}

static inline bool f32_al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static inline dim3 f32_rows_grid(int cols, int M) {
  return dim3((cols + 255) / 256, M < 65535 ? (M < 1 ? 1 : M) : 65535);
}

DLT_API int dlt_f32_swiglu_fwd(const float* gu, float* s, int M, int I, hipStream_t st) {
  if (I % 4 == 0 && f32_al16(gu) && f32_al16(s)) k_f32_swiglu_fwd<4><<<f32_rows_grid(I / 4, M), 256, 0, st>>>(gu, s, M, I);
  else k_f32_swiglu_fwd<1><<<f32_rows_grid(I, M), 256, 0, st>>>(gu, s, M, I);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_f32_swiglu_bwd(const float* gu, const float* da, float* dgu, float* s_out, int M, int I, hipStream_t st) {
  if (I % 4 == 0 && f32_al16(gu) && f32_al16(da) && f32_al16(dgu) && f32_al16(s_out)) k_f32_swiglu_bwd<4><<<f32_rows_grid(I / 4, M), 256, 0, st>>>(gu, da, dgu, s_out, M, I);
  else k_f32_swiglu_bwd<1><<<f32_rows_grid(I, M), 256, 0, st>>>(gu, da, dgu, s_out, M, I);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_f32_cross_entropy(float* logits, const long* targets, const long* n_valid, float* loss, int M, int Vp,
                                  int vocab, float grad_scale, hipStream_t st) {
  if (M <= 0) return 0;
  if (Vp % 4 == 0 && f32_al16(logits)) k_f32_ce_row<4><<<M, 256, 0, st>>>(logits, targets, n_valid, loss, Vp, vocab, grad_scale);
  else k_f32_ce_row<1><<<M, 256, 0, st>>>(logits, targets, n_valid, loss, Vp, vocab, grad_scale);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_f32_scale(const float* x, float* y, long n, const float* s, float mul, hipStream_t st) {
  k_f32_scale<<<f32_blocks(n), 256, 0, st>>>(x, y, n, s, mul);
  DLT_CHECK_LAUNCH();
}

// fwd: q/k/v strides (bs, hs, rs) in elements; o [B*S, nh*hd]; lse [B*nh, S]
DLT_API int dlt_f32_attn_fwd(const float* q, const float* k, const float* v, long bs, long hs, long rs, float* o,
                             float* lse, const uint32_t* mask, int B, int nh, int S, int hd, float scale, float dscale,
                             hipStream_t st) {
  F32Attn a{};
  a.q = q; a.k = k; a.v = v; a.bs = bs; a.hs = hs; a.rs = rs;
  a.out = o; a.lse = lse; a.mask = mask; a.B = B; a.nh = nh; a.S = S; a.scale = scale; a.dscale = dscale;
  const dim3 grid((S + F32_T - 1) / F32_T, B * nh);
  if (hd == 64) k_f32_attn_fwd<64><<<grid, 64, 0, st>>>(a);
  else if (hd == 128) k_f32_attn_fwd<128><<<grid, 64, 0, st>>>(a);
  else return -1;
  DLT_CHECK_LAUNCH();
}

// bwd: dq / dk / dv written with strides (gbs, ghs, grs) -- the packed dqkv or head-major
DLT_API int dlt_f32_attn_bwd(const float* q, const float* k, const float* v, long bs, long hs, long rs, const float* o,
                             const float* dO, const float* lse, const uint32_t* mask, float* delta, float* dq, float* dk,
                             float* dv, long gbs, long ghs, long grs, int B, int nh, int S, int hd, float scale,
                             float dscale, hipStream_t st) {
  F32Attn a{};
  a.q = q; a.k = k; a.v = v; a.bs = bs; a.hs = hs; a.rs = rs;
  a.dq = dq; a.dk = dk; a.dv = dv; a.gbs = gbs; a.ghs = ghs; a.grs = grs;
  a.o = o; a.dO = dO; a.lse = const_cast<float*>(lse); a.delta = delta; a.mask = mask;
  a.B = B; a.nh = nh; a.S = S; a.scale = scale; a.dscale = dscale;
  const dim3 grid((S + F32_T - 1) / F32_T, B * nh);
  if (hd == 64) {
    k_f32_attn_bwd_dq<64><<<grid, 64, 0, st>>>(a);
    k_f32_attn_bwd_dkdv<64><<<grid, 64, 0, st>>>(a);
  } else if (hd == 128) {
    k_f32_attn_bwd_dq<128><<<grid, 64, 0, st>>>(a);
    k_f32_attn_bwd_dkdv<128><<<grid, 64, 0, st>>>(a);
  } else {
    return -1;
  }
  DLT_CHECK_LAUNCH();
}

