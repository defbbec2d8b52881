// Weight-gradient GEMM:  C[N,K] (fp32, row-major) += A[M,N]^T . B[M,K]  (bf16 in).
//
// Every projection's wgrad has this shape (dW = dY^T X with the reduction over the
// B*S = 8192 token rows).  Both operands are stored with the reduction dim OUTER
// (M-major), the one layout the library heuristics handle badly on gfx950
// (180-700 TF/s measured, tools/wgrad_test.py).  Here both MFMA operands are read
// straight out of row-major LDS tiles with ds_read_b64_tr_b16 (hardware transpose),
// so no transposed copy of the activations or gradients is ever materialised, and
// the fp32 result is accumulated in place into the optimizer's main-grad buffer
// (fused "wgrad += " -- no bf16 round trip, no separate add kernel).
//
//   tile 128 (n) x 128 (k) per 256-thread workgroup, 4 waves as 2x2, each wave 64x64
//   = 2x2 v_mfma_f32_32x32x16_bf16 accumulators; reduction staged 64 rows at a time
//   through double-buffered LDS (register-staged global loads issued before the
//   MFMAs of the current stage); split over M (gridDim.z) when the output has too
//   few tiles to fill 256 CUs, combined with fp32 atomics (the L2-side atomic rate,
//   1.3 TB/s, bounds that combine; splits are chosen to keep it small).
#include "common.h"

#define WG_BN 128
#define WG_BK 128
#define WG_BM 64   // reduction rows per stage

typedef __attribute__((address_space(3))) shortx4_t lds_sx4_t;
typedef short sx8_t __attribute__((ext_vector_type(8)));

// LDS tile [64 rows][128 bf16] (256-B rows); 16-B chunk c of row r at chunk c ^ ((r & 3) << 2):
// the 4-row x 4-chunk footprint of one half-wave's transposed reads hits 16 distinct slots.
__device__ __forceinline__ int wg_off(int row, int col) {
  return row * 128 + ((((col >> 3) ^ ((row & 3) << 2))) << 3) + (col & 7);
}

// 32x32x16 operand fragment for rows (=reduction index) 16*s + 8*h + {0..7} and
// column c0 + (lane & 31): two transposed 4-row reads.
__device__ __forceinline__ bf16x8_t wg_frag(const bf16_t* T, int s, int c0, int lane) {
  const int h = lane >> 5, i = lane & 15;
  const int col = c0 + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const int r = 16 * s + 8 * h + (i >> 2);
  const shortx4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sx4_t*)(T + wg_off(r, col)));
  const shortx4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sx4_t*)(T + wg_off(r + 4, col)));
  sx8_t c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, c);
}

struct WgStage { u16x8 a[4], b[4]; };

__device__ __forceinline__ void wg_load(WgStage& st, const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                        int m0, int n0, int k0, int N, int K, int tid) {
  // 64 rows x 16 chunks (16 B) per operand = 1024 chunks -> 4 per thread
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + 256 * u;
    const int r = c >> 4, ch = c & 15;
    st.a[u] = *reinterpret_cast<const u16x8*>(A + (size_t)(m0 + r) * N + n0 + ch * 8);
    st.b[u] = *reinterpret_cast<const u16x8*>(B + (size_t)(m0 + r) * K + k0 + ch * 8);
  }
}

__device__ __forceinline__ void wg_store(const WgStage& st, bf16_t* TA, bf16_t* TB, int tid) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + 256 * u;
    const int r = c >> 4, ch = c & 15;
    *reinterpret_cast<u16x8*>(TA + wg_off(r, ch * 8)) = st.a[u];
    *reinterpret_cast<u16x8*>(TB + wg_off(r, ch * 8)) = st.b[u];
  }
}

__global__ __launch_bounds__(256, 2) void k_wgrad_gemm(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                       float* __restrict__ C, int M, int N, int K, int rows_per_split,
                                                       int use_atomics) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * WG_BM * 128];  // [buf][A|B][64][128]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid >> 1, wk = wid & 1;
  const int tiles_k = K / WG_BK;
  // XCD-aware: consecutive blocks (round-robin over the 8 XCDs) get tiles sharing B columns
  const int tile = blockIdx.x;
  const int tn = tile / tiles_k, tk = tile % tiles_k;
  const int n0 = tn * WG_BN, k0 = tk * WG_BK;
  const int m_begin = blockIdx.y * rows_per_split;
  const int m_end = min(M, m_begin + rows_per_split);
  const int nst = (m_end - m_begin) / WG_BM;

  floatx16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  WgStage st;
  if (nst > 0) {
    wg_load(st, A, B, m_begin, n0, k0, N, K, tid);
    wg_store(st, lds, lds + WG_BM * 128, tid);
  }
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nst;
    if (more) wg_load(st, A, B, m_begin + (s + 1) * WG_BM, n0, k0, N, K, tid);
    const bf16_t* TA = lds + cur * 2 * WG_BM * 128;
    const bf16_t* TB = TA + WG_BM * 128;
#pragma unroll
    for (int ks = 0; ks < WG_BM / 16; ++ks) {
      const bf16x8_t a0 = wg_frag(TA, ks, wn * 64, lane);
      const bf16x8_t a1 = wg_frag(TA, ks, wn * 64 + 32, lane);
      const bf16x8_t b0 = wg_frag(TB, ks, wk * 64, lane);
      const bf16x8_t b1 = wg_frag(TB, ks, wk * 64 + 32, lane);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      bf16_t* NA = lds + (cur ^ 1) * 2 * WG_BM * 128;
      wg_store(st, NA, NA + WG_BM * 128, tid);
    }
    __syncthreads();
  }
  // epilogue: D[n][k] with k = lane column, n = accumulator row
  const int h = lane >> 5;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int kc = k0 + wk * 64 + b * 32 + (lane & 31);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int nr = n0 + wn * 64 + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        float* p = C + (size_t)nr * K + kc;
        if (use_atomics) unsafeAtomicAdd(p, acc[a][b][i]);
        else *p += acc[a][b][i];
      }
    }
}

// C[N,K] += A[M,N]^T B[M,K]; returns -1 if the shape is not supported (caller falls back).
DLT_API int dlt_wgrad_gemm(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K, int splits,
                           hipStream_t st) {
  if (M % WG_BM || N % WG_BN || K % WG_BK || M <= 0) return -1;
  const int tiles = (N / WG_BN) * (K / WG_BK);
  if (splits <= 0) {  // aim for >= ~1 workgroup per CU; each extra split costs N*K*4 B of atomics
    splits = 1;
    while (tiles * splits < 200 && splits < 4 && (M / WG_BM) % (splits * 2) == 0 && M / (splits * 2) >= 1024)
      splits *= 2;
  }
  const int rows = ((M / WG_BM + splits - 1) / splits) * WG_BM;
  k_wgrad_gemm<<<dim3(tiles, splits), 256, 0, st>>>(A, B, C, M, N, K, rows, splits > 1 ? 1 : 0);
  DLT_CHECK_LAUNCH();
}
