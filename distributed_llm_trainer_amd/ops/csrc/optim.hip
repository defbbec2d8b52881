// Flat multi-tensor AdamW + global grad-norm for the fp32 master / bf16 shadow layout.
//
// Reference: torch.optim.AdamW(fused=True) over 110 tensors + clip_grad_norm_
// (foreach norm, host-visible scalar) + autocast re-casting every weight to bf16 each
// micro-step (ddp_trainer.py:229-234,347-356).  Here:
//  * k_sumsq + k_sum_partials: one pass over the flat fp32 grad buffer -> device
//    scalar (no host sync), bitwise reproducible;
//  * k_clip_coef: norm / clip coefficient computed ON DEVICE, folded with the DDP
//    1/world averaging into a single grad scale read by the AdamW kernel;
//  * k_adamw: decoupled weight decay + bias-corrected Adam on the flat buffer, also
//    writing the bf16 shadow weights the GEMMs consume.
#include "common.h"
#include <cstdlib>

// Deterministic two-stage sum of squares: every block writes its partial, one block
// adds the partials in a fixed order.  (A float atomicAdd per block made the sum --
// and so the clip coefficient -- depend on block completion order: DDP replicas
// drifted apart in the last bit, tests/test_distributed_gpu.py.)
constexpr int kSumsqMaxBlocks = 1024;

__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ x, int64_t n, float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n4 = n >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) acc += x[i] * x[i];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// *out += sum(part[0:nb]) in a fixed order (one block)
__global__ __launch_bounds__(256) void k_sum_partials(const float* __restrict__ part, int nb, float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out += (red[0] + red[1]) + (red[2] + red[3]);
}

// norm = sqrt(sumsq) * norm_mul;  coef = min(1, max_norm / (norm + 1e-6))  (clip_grad_norm_ semantics)
// out[0] = norm, out[1] = grad scale for AdamW = coef * scale_mul (max_norm <= 0 disables clipping)
__global__ void k_clip_coef(const float* __restrict__ sumsq, float* __restrict__ out, float norm_mul, float max_norm,
                            float scale_mul) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float norm = sqrtf(*sumsq) * norm_mul;
    float coef = 1.f;
    if (max_norm > 0.f) {
      coef = max_norm / (norm + 1e-6f);
      coef = coef < 1.f ? coef : 1.f;
    }
    out[0] = norm;
    out[1] = coef * scale_mul;
  }
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float lr, float b1, float b2, float eps,
                                          float wd, float step_size, float inv_bc2_sqrt) {
  p *= (1.f - lr * wd);
  m = m + (1.f - b1) * (g - m);  // lerp, as torch
  v = b2 * v + (1.f - b2) * g * g;
  const float denom = sqrtf(v) * inv_bc2_sqrt + eps;
  p -= step_size * m / denom;
}

// Streaming access for the optimizer pass: every byte is touched once per step (the
// 4.3 GB of p/g/m/v/shadow for GPT-2 small far exceed the 256 MB Infinity Cache), so
// nontemporal loads/stores keep it from evicting anything useful (DLT_ADAMW_NT=0: plain).
template <bool NTM>
__device__ __forceinline__ float4 ld4(const float* a, int64_t i) {
  if (NTM) {
    const float4* q = reinterpret_cast<const float4*>(a) + i;
    return make_float4(__builtin_nontemporal_load(&q->x), __builtin_nontemporal_load(&q->y),
                       __builtin_nontemporal_load(&q->z), __builtin_nontemporal_load(&q->w));
  }
  return reinterpret_cast<const float4*>(a)[i];
}
template <bool NTM>
__device__ __forceinline__ void st4(float* a, int64_t i, float4 x) {
  if (NTM) {
    float4* q = reinterpret_cast<float4*>(a) + i;
    __builtin_nontemporal_store(x.x, &q->x);
    __builtin_nontemporal_store(x.y, &q->y);
    __builtin_nontemporal_store(x.z, &q->z);
    __builtin_nontemporal_store(x.w, &q->w);
  } else {
    reinterpret_cast<float4*>(a)[i] = x;
  }
}

// 16-bit shadow conversion: bf16 (the fused engine) or fp16 (--mixed_precision fp16)
template <bool F16>
__device__ __forceinline__ uint16_t to_shadow(float x) {
  if constexpr (F16) {
    _Float16 h = (_Float16)x;
    return __builtin_bit_cast(uint16_t, h);
  } else {
    return f2bf(x);
  }
}

// ZG: the gradient is zeroed in the same pass (the lazy per-unit optimizer step of the
// flat store: the next micro-steps accumulate into it right after; no separate memset)
template <bool NTM, int OCC = 1, bool F16 = false, bool ZG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void k_adamw(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                               float* __restrict__ v, bf16_t* __restrict__ shadow, int64_t n, float lr,
                                               float b1, float b2, float eps, float wd, float step_size,
                                               float inv_bc2_sqrt, const float* __restrict__ gscale_ptr) {
  const float gs = gscale_ptr ? gscale_ptr[1] : 1.f;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto upd = [&](int64_t i, float4 pp, float4 gg, float4 mm, float4 vv) {
    adam_elem(pp.x, gg.x * gs, mm.x, vv.x, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt);
    adam_elem(pp.y, gg.y * gs, mm.y, vv.y, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt);
    adam_elem(pp.z, gg.z * gs, mm.z, vv.z, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt);
    adam_elem(pp.w, gg.w * gs, mm.w, vv.w, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt);
    st4<NTM>(p, i, pp);
    st4<NTM>(m, i, mm);
    st4<NTM>(v, i, vv);
    if (shadow) {
      u16x4 s;
      s.v[0] = to_shadow<F16>(pp.x); s.v[1] = to_shadow<F16>(pp.y);
      s.v[2] = to_shadow<F16>(pp.z); s.v[3] = to_shadow<F16>(pp.w);
      if (NTM) {
        const uint2 w = __builtin_bit_cast(uint2, s);
        uint32_t* q = reinterpret_cast<uint32_t*>(shadow) + 2 * i;
        __builtin_nontemporal_store(w.x, q);
        __builtin_nontemporal_store(w.y, q + 1);
      } else {
        reinterpret_cast<u16x4*>(shadow)[i] = s;
      }
    }
  };
  // two independent float4 groups per iteration: 8 loads in flight per thread
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const int64_t j = i + stride;
    const float4 p0 = ld4<NTM>(p, i), p1 = ld4<NTM>(p, j);
    const float4 g0 = ld4<NTM>(g, i), g1 = ld4<NTM>(g, j);
    const float4 m0 = ld4<NTM>(m, i), m1 = ld4<NTM>(m, j);
    const float4 v0 = ld4<NTM>(v, i), v1 = ld4<NTM>(v, j);
    if constexpr (ZG) {
      st4<NTM>(g, i, make_float4(0.f, 0.f, 0.f, 0.f));
      st4<NTM>(g, j, make_float4(0.f, 0.f, 0.f, 0.f));
    }
    upd(i, p0, g0, m0, v0);
    upd(j, p1, g1, m1, v1);
  }
  if (i < n4) {
    const float4 g0 = reinterpret_cast<const float4*>(g)[i];
    if constexpr (ZG) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    upd(i, reinterpret_cast<const float4*>(p)[i], g0, reinterpret_cast<const float4*>(m)[i],
        reinterpret_cast<const float4*>(v)[i]);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float pp = p[i], mm = m[i], vv = v[i];
      const float gi = g[i];
      if constexpr (ZG) g[i] = 0.f;
      adam_elem(pp, gi * gs, mm, vv, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt);
      p[i] = pp; m[i] = mm; v[i] = vv;
      if (shadow) shadow[i] = to_shadow<F16>(pp);
    }
  }
}

template <int HK = 0>
__global__ __launch_bounds__(256) void k_cast_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2h<HK>(x[i]);
}

static inline int flat_blocks(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

// part: device workspace of kSumsqMaxBlocks floats
DLT_API int dlt_sumsq(const float* x, int64_t n, float* part, float* out, hipStream_t st) {
  int nb = flat_blocks(n);
  if (nb > kSumsqMaxBlocks) nb = kSumsqMaxBlocks;
  k_sumsq<<<nb, 256, 0, st>>>(x, n, part);
  k_sum_partials<<<1, 256, 0, st>>>(part, nb, out);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_clip_coef(const float* sumsq, float* out, float norm_mul, float max_norm, float scale_mul,
                          hipStream_t st) {
  k_clip_coef<<<1, 64, 0, st>>>(sumsq, out, norm_mul, max_norm, scale_mul);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_adamw(float* p, float* g, float* m, float* v, bf16_t* shadow, int64_t n, float lr, float b1,
                      float b2, float eps, float wd, float step_size, float inv_bc2_sqrt, const float* gscale,
                      hipStream_t st) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  if (shadow && ((uintptr_t)shadow & 7)) return -1;
  static int nt = -1;
  if (nt < 0) {
    const char* e = getenv("DLT_ADAMW_NT");
    nt = (e && atoi(e) == 0) ? 0 : 1;
  }
  // eight waves per SIMD (63 instead of 67 VGPRs): 948 vs 1021 us for 152 M params,
  // step -0.1 ms in two same-box pairs; DLT_ADAMW_OCC=0 selects the unconstrained build
  static int occ = -1;
  if (occ < 0) {
    const char* e = getenv("DLT_ADAMW_OCC");
    occ = (e && atoi(e) == 0) ? 0 : 8;
  }
  if (nt && occ == 8)
    k_adamw<true, 8><<<flat_blocks(n), 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size,
                                                     inv_bc2_sqrt, gscale);
  else if (nt)
    k_adamw<true><<<flat_blocks(n), 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt,
                                                  gscale);
  else
    k_adamw<false><<<flat_blocks(n), 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt,
                                                   gscale);
  DLT_CHECK_LAUNCH();
}

// AdamW with an fp16 shadow (the engine's --mixed_precision fp16 weights)
DLT_API int dlt_adamw_f16(float* p, float* g, float* m, float* v, bf16_t* shadow, int64_t n, float lr, float b1,
                          float b2, float eps, float wd, float step_size, float inv_bc2_sqrt, const float* gscale,
                          hipStream_t st) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  if (shadow && ((uintptr_t)shadow & 7)) return -1;
  k_adamw<false, 1, true><<<flat_blocks(n), 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size,
                                                          inv_bc2_sqrt, gscale);
  DLT_CHECK_LAUNCH();
}

// AdamW with options (flags): bit 0 = fp16 shadow (else bf16 or none), bit 1 = zero the
// gradient in the same pass (the flat store's lazy per-unit step); bf16 runs the
// production build (nontemporal, eight waves per SIMD: dlt_adamw's defaults)
DLT_API int dlt_adamw_ex(float* p, float* g, float* m, float* v, bf16_t* shadow, int64_t n, float lr, float b1,
                         float b2, float eps, float wd, float step_size, float inv_bc2_sqrt, const float* gscale,
                         int flags, hipStream_t st) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  if (shadow && ((uintptr_t)shadow & 7)) return -1;
  const bool f16 = flags & 1, zg = flags & 2;
  const int nb = flat_blocks(n);
  if (f16 && zg)
    k_adamw<false, 1, true, true><<<nb, 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size,
                                                      inv_bc2_sqrt, gscale);
  else if (f16)
    k_adamw<false, 1, true><<<nb, 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size,
                                                inv_bc2_sqrt, gscale);
  else if (zg)
    k_adamw<true, 8, false, true><<<nb, 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size,
                                                      inv_bc2_sqrt, gscale);
  else
    k_adamw<true, 8><<<nb, 256, 0, st>>>(p, g, m, v, shadow, n, lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt,
                                         gscale);
  DLT_CHECK_LAUNCH();
}

// dst[i] += float(src[i]): the FSDP runtime folds a bf16 reduce-scatter output into the
// fp32 shard gradient in one pass (8 elements per lane, 16 B bf16 + 32 B fp32 loads).
template <int HK = 0>
__global__ __launch_bounds__(256) void k_add_bf16_f32(float* __restrict__ dst, const bf16_t* __restrict__ src,
                                                      int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const u16x8 s = reinterpret_cast<const u16x8*>(src)[i];
    float4* d = reinterpret_cast<float4*>(dst) + 2 * i;
    float4 a = d[0], b = d[1];
    a.x += h2f<HK>(s.v[0]); a.y += h2f<HK>(s.v[1]); a.z += h2f<HK>(s.v[2]); a.w += h2f<HK>(s.v[3]);
    b.x += h2f<HK>(s.v[4]); b.y += h2f<HK>(s.v[5]); b.z += h2f<HK>(s.v[6]); b.w += h2f<HK>(s.v[7]);
    d[0] = a;
    d[1] = b;
  }
}

// hk: src format (0 bf16, 1 fp16)
DLT_API int dlt_add_bf16_f32(float* dst, const bf16_t* src, int64_t n, int hk, hipStream_t st) {
  if (n % 8) return -1;
  DLT_HK_DISPATCH(hk, k_add_bf16_f32<HKC><<<flat_blocks(n / 2), 256, 0, st>>>(dst, src, n / 8));
  DLT_CHECK_LAUNCH();
}

// hk: output format (0 bf16, 1 fp16)
DLT_API int dlt_cast_bf16(const float* x, bf16_t* y, int64_t n, int hk, hipStream_t st) {
  DLT_HK_DISPATCH(hk, k_cast_bf16<HKC><<<flat_blocks(n * 4), 256, 0, st>>>(x, y, n));
  DLT_CHECK_LAUNCH();
}
