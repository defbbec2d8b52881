// Hand-written bf16 GEMM for the projection shapes:  C[M,N] = A[M,K] . B[N,K]^T
// (both operands K-contiguous, row-major; bf16 out, fp32 accumulate) -- the layout of
// every forward projection (y = x W^T) and, with a transposed weight copy, of the
// data-gradient GEMMs.
//
// CDNA4 structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * v_mfma_f32_32x32x16_bf16, operands straight from LDS with ds_read_b128;
//     "swapped" product D = B_frag . A_frag so each lane ends up owning one OUTPUT
//     ROW with 4 runs of 4 consecutive columns -> 8-byte stores in the epilogue;
//   * BK = 64 K-slices staged by global_load_lds_dwordx4 (LDS-DMA: no staging
//     registers) into a double-buffered image whose 16-B chunks are XOR-swizzled
//     (slot = chunk ^ ((row >> 1) & 7), applied on the SOURCE address because a DMA
//     wave-instruction writes 1 KiB lane-linearly) -> conflict-free b128 reads;
//   * the next slice's DMA is issued at the top of each step and retired by the
//     vmcnt(0) + barrier that ends it; the K loop is unrolled by two so both LDS
//     buffers are compile-time offsets;
//   * XCD-aware tile order: consecutive workgroups (which the dispatcher spreads over
//     the 8 XCDs) are remapped so each XCD owns a contiguous band of output tiles
//     that share A rows in its private L2 (bijective for any grid size).
// Tile configurations (BM x BN, waves WM x WN) are picked per shape by the planner
// in ops/gemm.py against the hipBLASLt candidates (fastest wins).
#include "common.h"

typedef __attribute__((address_space(3))) void* gt_lds_vptr_t;
typedef const __attribute__((address_space(1))) void* gt_gbl_cvptr_t;

#define GT_BK 64

__device__ __forceinline__ int gt_swz(int row, int chunk) { return row * GT_BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

// ROWS x 64 bf16 slice of a K-contiguous matrix into LDS (rows r0.., cols k0..k0+63).
template <int ROWS, int NW>
__device__ __forceinline__ void gt_stage(const bf16_t* __restrict__ G, int ld, int r0, int k0, bf16_t* T, int wid,
                                         int lane) {
  constexpr int PIECES = ROWS / 8;  // 1 KiB = 8 rows per wave-instruction
  static_assert(PIECES % NW == 0, "rows must split evenly over the waves");
#pragma unroll
  for (int j = 0; j < PIECES / NW; ++j) {
    const int rr = (wid * (PIECES / NW) + j) * 8;
    const int row = rr + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const bf16_t* g = G + (size_t)(r0 + row) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((gt_gbl_cvptr_t)g, (gt_lds_vptr_t)(T + rr * GT_BK), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8_t gt_frag(const bf16_t* T, int row, int s, int h) {
  return *reinterpret_cast<const bf16x8_t*>(T + gt_swz(row, 2 * s + h));
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_tn(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                          bf16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                          int ldc) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int STAGE = (BM + BN) * GT_BK;  // elements per LDS stage
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int h = lane >> 5, l32 = lane & 31;

  // XCD-aware bijective remap, then row-major tile order (tiles of one XCD share A rows)
  const int ntn = N / BN;
  const int nwg = (M / BM) * ntn;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;

  floatx16_t acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  const int nk = K / GT_BK;
  gt_stage<BM, NW>(A, lda, m0, 0, lds, wid, lane);
  gt_stage<BN, NW>(B, ldb, n0, 0, lds + BM * GT_BK, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto step = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
    if (kt + 1 < nk) {  // next slice into the other buffer (nobody reads it since the last barrier)
      bf16_t* Tn = lds + (BUF ^ 1) * STAGE;
      gt_stage<BM, NW>(A, lda, m0, (kt + 1) * GT_BK, Tn, wid, lane);
      gt_stage<BN, NW>(B, ldb, n0, (kt + 1) * GT_BK, Tn + BM * GT_BK, wid, lane);
    }
    const bf16_t* TA = lds + BUF * STAGE;
    const bf16_t* TB = TA + BM * GT_BK;
#pragma unroll
    for (int s = 0; s < GT_BK / 16; ++s) {
      bf16x8_t af[FM], bfr[FN];
#pragma unroll
      for (int b = 0; b < FM; ++b) af[b] = gt_frag(TA, wm * TM + b * 32 + l32, s, h);
#pragma unroll
      for (int a = 0; a < FN; ++a) bfr[a] = gt_frag(TB, wn * TN + a * 32 + l32, s, h);
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[a], af[b], acc[a][b], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
  }

  // epilogue: acc[a][b] = D[n][m]; this lane owns output row m, columns n in 4 runs of 4
#pragma unroll
  for (int b = 0; b < FM; ++b) {
    const int m = m0 + wm * TM + b * 32 + l32;
    bf16_t* crow = C + (size_t)m * ldc;
#pragma unroll
    for (int a = 0; a < FN; ++a) {
      const int nb = n0 + wn * TN + a * 32 + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w.v[e] = f2bf(acc[a][b][4 * g + e]);
        *reinterpret_cast<u16x4*>(crow + nb + 8 * g) = w;
      }
    }
  }
}

// cfg: 0 = 256x256 (8 waves 2x4), 1 = 256x128 (8 waves 4x2), 2 = 128x128 (4 waves 2x2),
//      3 = 128x64 (4 waves 2x2), 4 = 64x128 (4 waves 1x4)
// Returns -1 if the shape does not tile (the caller then uses the library GEMM).
DLT_API int dlt_gemm_tn(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb, int ldc,
                        int cfg, hipStream_t st) {
  if (K % GT_BK || M <= 0 || N <= 0 || (lda | ldb) % 8 || ldc % 4) return -1;
#define GT_LAUNCH(BM_, BN_, WM_, WN_)                                                                  \
  do {                                                                                                 \
    if (M % BM_ || N % BN_) return -1;                                                                 \
    k_gemm_tn<BM_, BN_, WM_, WN_><<<(M / BM_) * (N / BN_), 64 * WM_ * WN_, 0, st>>>(A, B, C, M, N, K, lda, \
                                                                                    ldb, ldc);         \
  } while (0)
  switch (cfg) {
    case 0: GT_LAUNCH(256, 256, 2, 4); break;
    case 1: GT_LAUNCH(256, 128, 4, 2); break;
    case 2: GT_LAUNCH(128, 128, 2, 2); break;
    case 3: GT_LAUNCH(128, 64, 2, 2); break;
    case 4: GT_LAUNCH(64, 128, 1, 4); break;
    default: return -1;
  }
#undef GT_LAUNCH
  DLT_CHECK_LAUNCH();
}
