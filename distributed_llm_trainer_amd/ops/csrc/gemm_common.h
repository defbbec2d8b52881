// Helpers shared by the hand-written GEMMs (gfx950): reduction-major ("token-major")
// operand tiles staged row-major by LDS-DMA with a per-row XOR chunk swizzle and read as
// MFMA fragments with ds_read_b64_tr_b16 (the hardware transpose).  Used by the weight-
// gradient kernel (gemm_wgrad.hip: both operands token-major) and the data-gradient form
// of the projection GEMM (gemm_bf16.hip BT = true: the weight W[Nred, Nout] is read as
// stored, reduction rows outermost).
#pragma once
#include "common.h"

typedef __attribute__((address_space(3))) void* gw_lds_vptr_t;
typedef short gw_sx8_t __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(1))) void* gw_gbl_cvptr_t;

// 16x16x32 MFMA on 16-bit operand fragments: HK = 0 bf16, 1 IEEE half (same shape, rate
// and fragment layout -- the staging and transposed reads move 16-bit words either way)
template <int HK>
__device__ __forceinline__ floatx4_t gw_mfma(const bf16x8_t& a, const bf16x8_t& b, const floatx4_t& c) {
  if constexpr (HK == 0) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
}

namespace {

constexpr int GW_BK = 64;
constexpr int GW_IMG_A = GW_BK * 128;  // elements of one A unit image / B0
constexpr int GW_IMG_B1 = GW_BK * 64;
constexpr int GW_BUF = 2 * GW_IMG_A + GW_IMG_A + GW_IMG_B1;  // A0, A1, B0, B1

// chunk swizzle of token row t: 256-byte rows (16 chunks) / 128-byte rows (8 chunks)
__device__ __forceinline__ int gw_v256(int t) { return (t & 3) | (((t >> 3) & 1) << 2); }
__device__ __forceinline__ int gw_v128(int t) { return ((t >> 1) & 1) | (((t >> 3) & 1) << 1); }

// image column -> column offset inside the tile's operand range
//   A unit q: image col j -> dW row wm*64 + q*32 + (j & 31), wm = j / 32
//   B0: image col j -> dW col (j / 64) * 96 + (j & 63);  B1: j -> (j / 32) * 96 + 64 + (j & 31)
__device__ __forceinline__ int gw_amap(int q, int j) { return (j >> 5) * 64 + q * 32 + (j & 31); }
//   (BN = 128 column tiles: B0 holds all 128 columns, image col j -> dW col j; no B1)
template <int BN = 192>
__device__ __forceinline__ int gw_b0map(int j) { return (j >> 6) * (BN / 2) + (j & 63); }
__device__ __forceinline__ int gw_b1map(int j) { return (j >> 5) * 96 + 64 + (j & 31); }

// LDS byte offset of (token row t, column col) in an image with 256- or 128-byte rows
template <int ROWB>
__device__ __forceinline__ uint32_t gw_off(int t, int col) {
  const int lc = col >> 3;
  const int pc = lc ^ (2 * (ROWB == 256 ? gw_v256(t) : gw_v128(t)));
  return (uint32_t)(t * ROWB + pc * 16 + (col & 7) * 2);
}

__device__ __forceinline__ shortx4_t gw_tr4(uint32_t addr) {
  shortx4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

// 16x16x32 operand fragment: tokens 32s + 8g + 0..7 (g = lane >> 4) of image column
// 16k + (lane & 15).  For those token rows the swizzle value v(t) is the same for every
// s and read half (t & 3 and bit 3 of t only depend on the lane), so a lane's address is
//   img + lbase + (32s + 4h) * ROWB + 32 * (k ^ v)
// with lbase / v per lane and 32 * (k ^ v) precomputed per k: the reads share a few base
// registers and take (32s + 4h) * ROWB as an immediate offset.
}  // namespace

template <int ROWB>
struct GwLane {
  uint32_t base;  // (8g + q) * ROWB + 16 * ((i >> 1) & 1) + 8 * (i & 1)
  int v;
  __device__ __forceinline__ void init(int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2;
    const int t = 8 * g + q;
    base = (uint32_t)(t * ROWB + 16 * ((i >> 1) & 1) + 8 * (i & 1));
    v = ROWB == 256 ? gw_v256(t) : gw_v128(t);
  }
  __device__ __forceinline__ uint32_t koff(int k) const { return (uint32_t)(32 * (k ^ v)); }
};

template <int ROWB>
__device__ __forceinline__ bf16x8_t gw_frag(uint32_t img_lane_k, int s) {
  const shortx4_t a = gw_tr4(img_lane_k + (uint32_t)(32 * s) * ROWB);
  const shortx4_t b = gw_tr4(img_lane_k + (uint32_t)(32 * s + 4) * ROWB);
  gw_sx8_t c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, c);
}

