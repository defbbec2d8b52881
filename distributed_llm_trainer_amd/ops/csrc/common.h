// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this framework.
//
// Conventions
//  * wave = 64 lanes; every block size is a multiple of 64.
//  * bf16 tensors are handled as raw 16-bit words and moved in 16-byte vectors
//    (8 x bf16 per lane) -- hipcc does not vectorise scalar bf16 loads.
//  * f32 -> bf16 uses the compiler cast (v_cvt_pk_bf16_f32, RNE, NaN-preserving).
//  * Dropout randomness: lowbias32 hash of (key ^ pair_index); one hash gives 16
//    bits to each of two neighbouring elements (see ops/rng.py for the contract).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DLT_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef float floatx16_t __attribute__((ext_vector_type(16)));
typedef short shortx4_t __attribute__((ext_vector_type(4)));

struct alignas(16) u16x8 { uint16_t v[8]; };
struct alignas(8) u16x4 { uint16_t v[4]; };

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// 16-bit activation formats.  HK = 0: bf16 (the default compute dtype); HK = 1: fp16
// (--mixed_precision fp16: the same kernels instantiated for IEEE half, RNE casts).
// Kernels that move activations as raw 16-bit words take HK as a template parameter and
// their launchers an `hk` argument (0 / 1).
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
template <int HK>
__device__ __forceinline__ float h2f(uint16_t u) {
  if constexpr (HK == 0) return __uint_as_float(((uint32_t)u) << 16);
  else return (float)__builtin_bit_cast(_Float16, u);
}
template <int HK>
__device__ __forceinline__ uint16_t f2h(float f) {
  if constexpr (HK == 0) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
  } else {
    return __builtin_bit_cast(uint16_t, (_Float16)f);
  }
}
// launcher helper: run F<0> or F<1> by the runtime format
#define DLT_HK_DISPATCH(hk, ...) \
  do {                           \
    if ((hk) == 1) {             \
      constexpr int HKC = 1;     \
      __VA_ARGS__;               \
    } else {                     \
      constexpr int HKC = 0;     \
      __VA_ARGS__;               \
    }                            \
  } while (0)

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// 16 random bits for flat element index `idx` under `key`.
__device__ __forceinline__ uint32_t drop_bits(uint32_t key, uint64_t idx) {
  uint32_t h = lowbias32(key ^ (uint32_t)(idx >> 1));
  return (idx & 1) ? (h >> 16) : (h & 0xffffu);
}

// sigmoid with the hardware reciprocal (v_rcp_f32, 1 ulp): the IEEE division hipcc
// emits for `1.f / x` is a ~10-instruction sequence, which dominated the SwiGLU GEMM
// epilogue.  Every SwiGLU kernel uses this one so the fused and unfused paths agree.
__device__ __forceinline__ float dlt_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define DLT_CHECK_LAUNCH() return (int)hipGetLastError()

// Device-side bounds checks, compiled in only for the debug library
// (`python -m distributed_llm_trainer_amd.ops.build --debug` -> _dlt_kernels_debug.so,
// selected at run time with DLT_KERNEL_DEBUG=1): a failed check prints the condition
// and traps the wave, so a bad token id or target stops at the faulting kernel instead
// of silently reading another row (XNACK is off: out-of-range reads inside the
// allocation do not fault).
#ifdef DLT_DEBUG
#define DLT_DASSERT(cond)                                                        \
  do {                                                                           \
    if (!(cond)) {                                                               \
      printf("DLT_DASSERT failed %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
      __builtin_trap();                                                          \
    }                                                                            \
  } while (0)
#else
#define DLT_DASSERT(cond) ((void)0)
#endif
