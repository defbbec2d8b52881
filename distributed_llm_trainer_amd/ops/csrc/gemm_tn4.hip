// Four-wave, one-tile-per-workgroup bf16 "TN" GEMM for the forward projections
// (gfx950 / MI355X):   C[M,N] = A[M,K] . B[N,K]^T   (both operands K-contiguous, fp32
// accumulate) -- the q/k/v, o, gate/up, down and lm_head forwards of
// /root/reference/src/models/gpt.py:185-187, :239, :278-281, :447.
//
// Why a second forward GEMM (round 5): the persistent 8-wave k_gemm_bf16 (gemm_bf16.hip)
// beats hipBLASLt on qkv / o / down in isolation but loses in the two-chain training step,
// where it shares every CU with the other chain's attention / norm kernels.  Its 8 waves
// own 64 x 96 outputs each, so one 256 x 192 tile reads (64 + 96) x 8 rows of fragments
// per 32-deep k-step: 0.67 LDS instructions per MFMA (PMC, profiles/r4_pmc_counters.md)
// against hipBLASLt's 0.25, and the LDS pipe is exactly what the co-running attention
// kernels use most.  This kernel takes the library kernel's shape instead:
//   * 256 x 256 tile, 256 threads = 4 waves as 2 (M) x 2 (N), each wave 128 x 128 outputs
//     = 8 x 8 tiles of v_mfma_f32_16x16x32_bf16 (256 accumulator registers; one wave per
//     SIMD with the whole 512-register file): 16 ds_read_b128 per 64 MFMAs (0.25 / MFMA);
//   * one tile per workgroup (grid = tile count), so the dispatcher hands CUs back to the
//     other chain tile by tile; XCD-aware tile order (each XCD walks a contiguous range of
//     row-major tiles: one A row panel, all of B, through its own L2);
//   * BK = 32 stages by LDS-DMA (global_load_lds_dwordx4, SGPR base + 32-bit lane offsets;
//     a stage row is 64 bytes, so the 16 rows of a fragment read are one contiguous,
//     conflict-free KiB), a ring of 4 stages: one counted wait + one barrier per stage,
//     placed between the two halves of the stage's MFMAs, so the next stage's fragment
//     reads overlap the second half and the barrier never drains the MFMA pipe; the DMA
//     of the stage 4 ahead is issued right after it (a 2-stage BK = 64 ring with the
//     barrier at the stage boundary ran 30-60 % behind hipBLASLt);
//   * epilogue through LDS: each wave writes its 128 x 128 bf16 block (swapped product
//     D = B.A^T, so a lane holds 4 consecutive columns of one row: one 8-byte LDS write per
//     16 x 16 tile), then stores whole 256-byte row runs with 16-byte global stores.
//
// Requirements (launcher-checked): M % 256 == 0, K % 32 == 0, N % 8 == 0 (a ragged last
// column tile clamps its B rows and masks its stores), 16-byte aligned rows.
// HK: operand / output format, 0 = bf16, 1 = IEEE half (--mixed_precision fp16).
#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int T4_BM = 256, T4_BN = 256;
constexpr int T4_CROW = 136;                 // epilogue staging row (elements; 8 pad)
constexpr int T4_CSTG = 128 * T4_CROW;       // per-wave staging block (elements)

// Stage geometry: BK = 32 (64-byte rows, no swizzle: the 16 rows of a fragment read are
// one contiguous KiB) in a ring of 4, or BK = 64 (128-byte rows, chunk c of row r at
// c ^ ((r >> 1) & 7): conflict-free) in a ring of 2 -- 128 KiB of LDS either way.
template <int BK>
struct T4Cfg {
  static constexpr int NBUF = BK == 32 ? 4 : 2;
  static constexpr int IMG = T4_BM * BK;     // elements of one operand image
  static constexpr int STAGE = 2 * IMG;
  static constexpr int CPR = BK / 8;         // 16-byte chunks per row
  static constexpr int RPI = 64 / CPR;       // rows per DMA instruction (1 KiB)
  static constexpr int NI = 64 / RPI;        // DMA instructions per wave per operand
  static constexpr int PIECES = 2 * NI;      // per wave per stage
  static constexpr int SPS = BK / 32;        // 32-deep k-steps per stage
  static constexpr int LDS = (NBUF * STAGE > 4 * T4_CSTG) ? NBUF * STAGE : 4 * T4_CSTG;
  static __device__ __forceinline__ int off(int row, int chunk) {
    if constexpr (BK == 32) return row * BK + (chunk << 3);
    else return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3);
  }
};

// One LDS-DMA piece (64 lanes x 16 B -> 1 KiB at lds_dst), SGPR base + 32-bit lane byte
// offset.  Issued from inline asm, so the compiler's wait pass neither sees nor waits for
// it: the kernel retires the pieces itself (counted s_waitcnt vmcnt + barrier per stage).
__device__ __forceinline__ void t4_dma(const void* gbase, uint32_t voff, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(gbase), "s"(m0)
               : "memory", "m0");
}

// this wave's DMA pieces older than the newest n retired
__device__ __forceinline__ void t4_vmwait(int n) {
  if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

typedef __bf16 t4_bf16x4_t __attribute__((ext_vector_type(4)));
typedef _Float16 t4_f16x4_t __attribute__((ext_vector_type(4)));
template <int HK>
__device__ __forceinline__ uint2 t4_pack(const floatx4_t& v) {
  if constexpr (HK == 0) return __builtin_bit_cast(uint2, __builtin_convertvector(v, t4_bf16x4_t));
  else return __builtin_bit_cast(uint2, __builtin_convertvector(v, t4_f16x4_t));
}

}  // namespace

template <int HK, int BK>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_gemm_tn4(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, bf16_t* __restrict__ C, int M, int N, int K, int lda,
    int ldb, int ldc) {
  using Cf = T4Cfg<BK>;
  __shared__ __attribute__((aligned(16))) bf16_t lds[Cf::LDS];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid & 1, wn = wid >> 1;
  const int l16 = lane & 15, lq = lane >> 4;

  // tile: XCD x (= block id mod 8, the dispatcher's round-robin) walks a contiguous range
  // of the row-major tile order (bijective for any grid size)
  const int ntn = (N + T4_BN - 1) / T4_BN;
  const int nb = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = t / ntn, tn = t - tm * ntn;
  const int m0 = tm * T4_BM, n0 = tn * T4_BN;

  // per-lane DMA byte offsets: wave w stages rows w*64 + RPI*j + lane / CPR of both
  // images; the lane's physical slot p = lane % CPR holds global chunk p (BK = 32) or
  // p ^ ((row >> 1) & 7) (BK = 64)
  uint32_t aoff[Cf::NI], boff[Cf::NI];
#pragma unroll
  for (int j = 0; j < Cf::NI; ++j) {
    const int row = wid * 64 + Cf::RPI * j + lane / Cf::CPR;
    const int p = lane % Cf::CPR;
    const int c = BK == 32 ? p : (p ^ ((row >> 1) & 7));
    aoff[j] = (uint32_t)(row * lda + c * 8) * 2u;
    const int brow = min(n0 + row, N - 1) - n0;  // ragged last column tile: clamp
    boff[j] = (uint32_t)(brow * ldb + c * 8) * 2u;
  }
  const bf16_t* Ab = A + (size_t)m0 * lda;
  const bf16_t* Bb = B + (size_t)n0 * ldb;
  auto stage = [&](int st, int buf) {
    bf16_t* la = lds + buf * Cf::STAGE;
    bf16_t* lb = la + Cf::IMG;
    const bf16_t* ga = Ab + st * BK;
    const bf16_t* gb = Bb + st * BK;
#pragma unroll
    for (int j = 0; j < Cf::NI; ++j) t4_dma(ga, aoff[j], la + (wid * 64 + Cf::RPI * j) * BK);
#pragma unroll
    for (int j = 0; j < Cf::NI; ++j) t4_dma(gb, boff[j], lb + (wid * 64 + Cf::RPI * j) * BK);
  };

  floatx4_t acc[8][8];  // [n-tile][m-tile]: D = B_tile . A_tile^T
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};

  // The k loop runs over 32-deep k-steps j; a k-step's fragments are read into registers
  // during k-step j - 1, so k-step j is: MFMAs of n-tiles 0-3 | [last k-step of its stage:
  // wait for the next stage, barrier, DMA of the stage NBUF ahead into this stage's buffer
  // (every wave has read it: its last fragments are in registers)] reads of k-step
  // j + 1's fragments | MFMAs of n-tiles 4-7, which cover the read latency -- the
  // barrier never drains the MFMA pipe.  Fragment registers alternate between two sets
  // (the loop is unrolled by two).
  const int ns = K / BK, nks = K / 32;
#pragma unroll
  for (int st = 0; st < Cf::NBUF; ++st)
    if (st < ns) stage(st, st);
  // at the end of stage st: stages <= min(st - 1 + NBUF, ns - 1) are issued (the prologue's
  // NBUF plus one per finished stage), stage st + 1 must have landed -- the younger ones
  // may stay in flight
  auto wait_next = [&](int st) {
    t4_vmwait((min(st - 1 + Cf::NBUF, ns - 1) - (st + 1)) * Cf::PIECES);
    __syncthreads();
  };
  auto read_frags = [&](int j, bf16x8_t (&fa)[8], bf16x8_t (&fb)[8]) {
    const int st = j / Cf::SPS, ks = j % Cf::SPS;
    const bf16_t* la = lds + (st % Cf::NBUF) * Cf::STAGE;
    const bf16_t* lb = la + Cf::IMG;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fa[i] = *reinterpret_cast<const bf16x8_t*>(la + Cf::off(wm * 128 + 16 * i + l16, 4 * ks + lq));
      fb[i] = *reinterpret_cast<const bf16x8_t*>(lb + Cf::off(wn * 128 + 16 * i + l16, 4 * ks + lq));
    }
  };
  // prologue: stage 0 landed (NBUF - 1 younger stages may be in flight)
  t4_vmwait((min(Cf::NBUF, ns) - 1) * Cf::PIECES);
  __syncthreads();
  bf16x8_t af[2][8], bf[2][8];
  read_frags(0, af[0], bf[0]);
  auto kstep = [&](int j, bf16x8_t (&fa)[8], bf16x8_t (&fb)[8], bf16x8_t (&ga)[8], bf16x8_t (&gb)[8]) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int m = 0; m < 8; ++m) acc[n][m] = gw_mfma<HK>(fb[n], fa[m], acc[n][m]);
    if (j + 1 < nks) {
      const int st = j / Cf::SPS;
      if (j % Cf::SPS == Cf::SPS - 1) {
        wait_next(st);
        if (st + Cf::NBUF < ns) stage(st + Cf::NBUF, st % Cf::NBUF);
      }
      read_frags(j + 1, ga, gb);
    }
#pragma unroll
    for (int n = 4; n < 8; ++n)
#pragma unroll
      for (int m = 0; m < 8; ++m) acc[n][m] = gw_mfma<HK>(fb[n], fa[m], acc[n][m]);
  };
  __builtin_amdgcn_s_setprio(1);
#pragma unroll 1
  for (int j = 0; j < nks; j += 2) {
    kstep(j, af[0], bf[0], af[1], bf[1]);
    if (j + 1 < nks) kstep(j + 1, af[1], bf[1], af[0], bf[0]);
  }
  __builtin_amdgcn_s_setprio(0);

  // epilogue: lane holds C[m0 + wm*128 + 16m + l16][n0 + wn*128 + 16n + 4lq + 0..3]
  __syncthreads();  // every wave is done with the operand buffers the staging reuses
  bf16_t* stg = lds + wid * T4_CSTG;
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int m = 0; m < 8; ++m)
      *reinterpret_cast<uint2*>(stg + (16 * m + l16) * T4_CROW + 16 * n + 4 * lq) = t4_pack<HK>(acc[n][m]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own block only: no barrier needed
  const int ch = lane & 15;
  const int ncol = n0 + wn * 128 + ch * 8;
  bf16_t* crow = C + (size_t)(m0 + wm * 128 + (lane >> 4)) * ldc + ncol;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    const int row = 4 * i + (lane >> 4);
    const uint4 v = *reinterpret_cast<const uint4*>(stg + row * T4_CROW + ch * 8);
    if (ncol < N) *reinterpret_cast<uint4*>(crow + (size_t)(4 * i) * ldc) = v;
  }
}

#include <cstdlib>
// stage depth: DLT_TN4_BK=32 (ring of 4, default) | 64 (ring of 2)
static int t4_bk() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DLT_TN4_BK");
    v = (e && atoi(e) == 64) ? 64 : 32;
  }
  return v;
}

DLT_API int dlt_gemm_tn4(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb, int ldc,
                         int hk, hipStream_t st) {
  const int bk = t4_bk();
  if (M <= 0 || N <= 0 || K <= 0 || M % T4_BM || K % bk || N % 8 || lda % 8 || ldb % 8 || ldc % 8 || lda < K ||
      ldb < K || ldc < N)
    return -1;
  const long tiles = (long)(M / T4_BM) * ((N + T4_BN - 1) / T4_BN);
  if (tiles > 0x7fffffff) return -1;
  if (bk == 64)
    DLT_HK_DISPATCH(hk, k_gemm_tn4<HKC, 64><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc));
  else
    DLT_HK_DISPATCH(hk, k_gemm_tn4<HKC, 32><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc));
  DLT_CHECK_LAUNCH();
}
