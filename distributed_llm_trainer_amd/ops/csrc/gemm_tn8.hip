// 256x256 "8-phase" bf16 GEMM for the large projection shapes:
//   C[M,N] = A[M,K] . B[N,K]^T   (both operands K-contiguous, bf16 out, fp32 accumulate)
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template"), written for this
// framework's shapes (K = 768 / 3072 projections, the 50k-column lm_head):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 output block,
//     i.e. 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 = 128 fp32 accumulators per lane.
//   * BK = 64.  One K-tile of A (256 x 64) and B (256 x 64) lives in a 64 KB LDS
//     buffer; two buffers (even / odd K-tiles) = 128 KB, all in ONE __shared__ array.
//   * Each K-tile is consumed in 4 phases, one per 64 x 32 quadrant of every wave's
//     block (16 MFMAs each): q0 = (rows 0-63, cols 0-31) reads A-half 0 and B-half 0,
//     q1 = (0-63, 32-63) reads B-half 1, q2 = (64-127, 32-63) reads A-half 1,
//     q3 = (64-127, 0-31) reuses registers only.  The "halves" are the staging
//     units: 128 rows x 64 k = 16 KB = 2 global_load_lds_dwordx4 per wave.
//   * Staging: one unit per phase, LDS-DMA (no staging registers), source-side XOR
//     swizzle (16-B chunk ^= (row >> 1) & 7) -> conflict-free ds_read_b128 for the
//     16x16x32 fragment pattern.  A unit is restaged >= 2 phases after its last read
//     (WAR), and each buffer is retired by a COUNTED vmcnt(4) (2 units still in flight
//     across the barrier) one phase before it is read (RAW) -- never vmcnt(0) in the
//     steady state, raw s_barrier (no __syncthreads, whose fence would drain the DMA).
//   * Waves 4-7 (second M half) run one barrier behind waves 0-3, so on every SIMD one
//     wave's MFMA segment overlaps its partner's LDS-read/DMA-issue segment; the MFMA
//     clusters run at s_setprio(1).
//   * XCD-aware bijective tile order (consecutive tiles of one XCD share A rows in
//     its private L2).
// Requirements (checked by the launcher): M % 256 == 0, N % 256 == 0, K % 128 == 0,
// 16-B aligned rows.  The planner (ops/gemm.py) races it against hipBLASLt per shape.
#include "common.h"

typedef __attribute__((address_space(3))) void* g8_lds_vptr_t;
typedef const __attribute__((address_space(1))) void* g8_gbl_cvptr_t;

namespace {

constexpr int G8_BK = 64;
constexpr int G8_TILE = 256 * G8_BK;        // elements of one operand tile image
constexpr int G8_BUF = 2 * G8_TILE;         // A image + B image

__device__ __forceinline__ int g8_swz(int row, int chunk) { return row * G8_BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

// Tile rows covered by 8-row group g (0..15) of a staging unit.
//   A unit qm: rows {0..63} u {128..191} (qm = 0) or {64..127} u {192..255} (qm = 1)
//   B unit qn: rows {c*64 + qn*32 + 0..31 : c = 0..3}
template <bool IS_A>
__device__ __forceinline__ int g8_group_row(int q, int g) {
  if (IS_A) return (g >> 3) * 128 + q * 64 + (g & 7) * 8;
  return (g >> 2) * 64 + q * 32 + (g & 3) * 8;
}

// Per-lane element offset (inside a K-tile, relative to the tile's first row) of the
// j-th LDS-DMA of staging unit q -- precomputed once, so the loop only adds a
// wave-uniform base (saddr form, one 32-bit VGPR per DMA).
template <bool IS_A>
__device__ __forceinline__ uint32_t g8_src_off(int ld, int q, int j, int wid, int lane) {
  const int row = g8_group_row<IS_A>(q, wid * 2 + j) + (lane >> 3);
  const int c = (lane & 7) ^ ((row >> 1) & 7);
  return (uint32_t)(row * ld + c * 8) * 2u;  // bytes
}

// Issue one staging unit (2 LDS-DMA instructions per wave) from the uniform base `g`
// (row r0, column kt*BK of the operand).
template <bool IS_A>
__device__ __forceinline__ void g8_stage(const bf16_t* g, const uint32_t (&off)[2], int q, bf16_t* img, int wid) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rb = g8_group_row<IS_A>(q, wid * 2 + j);
    __builtin_amdgcn_global_load_lds((g8_gbl_cvptr_t)((const char*)g + off[j]), (g8_lds_vptr_t)(img + rb * G8_BK), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8_t g8_frag(const bf16_t* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(img + g8_swz(row, chunk));
}

}  // namespace

// Epilogues: EPI_STORE writes C = A.B^T (bf16).  EPI_SWIGLU_BWD is the SwiGLU backward
// fused onto the down-projection data gradient: the tile of ds = dd . Wdown (C, never
// stored) meets the saved gate/up activations and only dgu is written,
//   dg = ds * u * sig(g) * (1 + g (1 - sig(g))),   du = ds * g * sig(g)
// (gu / dgu: [M, 2I] rows, gate in columns [0, I), up in [I, 2I); N == I) -- the math
// of k_swiglu_bwd (elementwise.hip) on the fp32 accumulator instead of a bf16 ds.
// It removes the ds round trip (write + read of [M, I] bf16) and one launch, but at one
// workgroup per CU the epilogue's gu/dgu traffic (4x the plain tile store) cannot
// overlap another tile's main loop: measured 203 us vs 168 us for hipBLASLt + the
// SwiGLU kernel at M = 16384 (plain tn8 92 us), so the planner's race
// (HipGemm.dgrad_swiglu) keeps the unfused pair on MI355X today.
enum { EPI_STORE = 0, EPI_SWIGLU_BWD = 1 };

__device__ __forceinline__ float g8_sigmoid(float x) { return 1.f / (1.f + __expf(-x)); }

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_tn8(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                     bf16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                     int ldc, const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
                                                     int I) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * G8_BUF];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int l16 = lane & 15, lq = lane >> 4;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD), row-major tile order
  const int ntn = N >> 8;
  const int nwg = (M >> 8) * ntn;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (wg / ntn) << 8, n0 = (wg % ntn) << 8;

  bf16_t* const A0 = lds;                 // buffer 0: A image, B image
  bf16_t* const B0i = lds + G8_TILE;
  bf16_t* const A1 = lds + G8_BUF;        // buffer 1
  bf16_t* const B1i = lds + G8_BUF + G8_TILE;

  floatx4_t acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / G8_BK;  // even, >= 2
  uint32_t oa[2][2], ob[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      oa[q][j] = g8_src_off<true>(lda, q, j, wid, lane);
      ob[q][j] = g8_src_off<false>(ldb, q, j, wid, lane);
    }
  const bf16_t* const Ab = A + (size_t)m0 * lda;
  const bf16_t* const Bb = B + (size_t)n0 * ldb;
#define G8A(kt, q, img) g8_stage<true>(Ab + (kt) * G8_BK, oa[q], q, img, wid)
#define G8B(kt, q, img) g8_stage<false>(Bb + (kt) * G8_BK, ob[q], q, img, wid)

  // prologue: the state at the top of iteration 0 -- K-tile 0 complete in buffer 0,
  // A/B unit 0 of K-tile 1 in flight (their steady-state slots are phases 7 and 8)
  G8A(0, 0, A0);
  G8B(0, 0, B0i);
  G8B(0, 1, B0i);
  G8A(0, 1, A0);
  G8A(1, 0, A1);
  G8B(1, 0, B1i);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 run one barrier behind

  // fragments: A rows of quadrant-half qm, B rows of quadrant-half qn, k-substeps s
  bf16x8_t fa[4][2], fb0[2][2], fb1[2][2];
  const int arow = wr * 128 + l16;  // + qm*64 + mt*16
  const int brow = wc * 64 + l16;   // + qn*32 + nt*16

  auto read_a = [&](const bf16_t* img, int qm) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[mt][s] = g8_frag(img, arow + qm * 64 + mt * 16, s * 4 + lq);
  };
  auto read_b = [&](const bf16_t* img, int qn, bf16x8_t (&fb)[2][2]) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb[nt][s] = g8_frag(img, brow + qn * 32 + nt * 16, s * 4 + lq);
  };
  // 16 MFMAs: quadrant (qm, qn) += fb(qn) x fa  (swapped product: D[n][m], so a lane
  // owns one output row m and 4 consecutive columns n -> 8-byte stores)
  auto mma = [&](int qm, int qn, bf16x8_t (&fb)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[qn * 2 + nt][qm * 4 + mt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt][s], fa[mt][s], acc[qn * 2 + nt][qm * 4 + mt], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  for (int kt = 0; kt < nk; kt += 2) {
    const bool more = kt + 2 < nk;  // K-tiles kt+2 / kt+3 exist (nk even)
    // ---- phase 1: buffer 0, q0 ; stage B-half 1 of tile kt+1
    read_b(B0i, 0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(A0, 0);
    G8B(kt + 1, 1, B1i);
    __builtin_amdgcn_s_barrier();
    mma(0, 0, fb0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: q1 ; stage A-half 1 of tile kt+1
    read_b(B0i, 1, fb1);
    G8A(kt + 1, 1, A1);
    __builtin_amdgcn_s_barrier();
    mma(0, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: q2 ; restage A-half 0 of buffer 0 with tile kt+2
    read_a(A0, 1);
    if (more) G8A(kt + 2, 0, A0);
    __builtin_amdgcn_s_barrier();
    mma(1, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: q3 (registers only) ; B-half 0 of tile kt+2 ; retire tile kt+1
    if (more) {
      G8B(kt + 2, 0, B0i);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    mma(1, 0, fb0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 5: buffer 1, q0 ; B-half 1 of tile kt+2
    read_b(B1i, 0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(A1, 0);
    if (more) G8B(kt + 2, 1, B0i);
    __builtin_amdgcn_s_barrier();
    mma(0, 0, fb0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 6: q1 ; A-half 1 of tile kt+2
    read_b(B1i, 1, fb1);
    if (more) G8A(kt + 2, 1, A0);
    __builtin_amdgcn_s_barrier();
    mma(0, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 7: q2 ; A-half 0 of tile kt+3
    read_a(A1, 1);
    if (more) G8A(kt + 3, 0, A1);
    __builtin_amdgcn_s_barrier();
    mma(1, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 8: q3 ; B-half 0 of tile kt+3 ; retire tile kt+2
    if (more) {
      G8B(kt + 3, 0, B1i);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    mma(1, 0, fb0);
    __builtin_amdgcn_s_barrier();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts for both halves
#undef G8A
#undef G8B

  // epilogue: acc[nt][mt] = D[n][m] of a 16x16 tile; lane owns row m = l16, columns
  // 4*lq .. 4*lq+3
  if constexpr (EPI == EPI_STORE) {
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      bf16_t* crow = C + (size_t)(m0 + wr * 128 + mt * 16 + l16) * ldc + n0 + wc * 64 + lq * 4;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w.v[e] = f2bf(acc[nt][mt][e]);
        *reinterpret_cast<u16x4*>(crow + nt * 16) = w;
      }
    }
  } else {
    const size_t ld2 = 2 * (size_t)I;
    const int c0 = n0 + wc * 64 + lq * 4;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const size_t row = (size_t)(m0 + wr * 128 + mt * 16 + l16) * ld2;
      u16x4 gcur[4], ucur[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {  // all loads of the row block first
        gcur[nt] = *reinterpret_cast<const u16x4*>(gu + row + c0 + nt * 16);
        ucur[nt] = *reinterpret_cast<const u16x4*>(gu + row + I + c0 + nt * 16);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        u16x4 og, ou;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float g = bf2f(gcur[nt].v[e]), u = bf2f(ucur[nt].v[e]), d = acc[nt][mt][e];
          const float sg = g8_sigmoid(g);
          og.v[e] = f2bf(d * u * sg * (1.f + g * (1.f - sg)));
          ou.v[e] = f2bf(d * g * sg);
        }
        *reinterpret_cast<u16x4*>(dgu + row + c0 + nt * 16) = og;
        *reinterpret_cast<u16x4*>(dgu + row + I + c0 + nt * 16) = ou;
      }
    }
  }
}

DLT_API int dlt_gemm_tn8(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb, int ldc,
                         hipStream_t st) {
  if (M <= 0 || N <= 0 || M % 256 || N % 256 || K % 128 || K < 128 || (lda | ldb) % 8 || ldc % 4) return -1;
  k_gemm_tn8<EPI_STORE><<<(M / 256) * (N / 256), 512, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, nullptr, nullptr, 0);
  DLT_CHECK_LAUNCH();
}

// dgu[M, 2I] = swiglu_bwd(gu, dd . Wdown) with B = Wdown^T [I, K] (K-contiguous rows):
// the down-projection data gradient and the SwiGLU backward in one kernel.
DLT_API int dlt_gemm_tn8_swiglu_bwd(const bf16_t* A, const bf16_t* B, const bf16_t* gu, bf16_t* dgu, int M, int I,
                                    int K, int lda, int ldb, hipStream_t st) {
  if (M <= 0 || I <= 0 || M % 256 || I % 256 || K % 128 || K < 128 || (lda | ldb) % 8) return -1;
  k_gemm_tn8<EPI_SWIGLU_BWD><<<(M / 256) * (I / 256), 512, 0, st>>>(A, B, nullptr, M, I, K, lda, ldb, 0, gu, dgu, I);
  DLT_CHECK_LAUNCH();
}
