// One-tile-per-workgroup bf16 "TN" GEMM for the forward projections (gfx950 / MI355X):   C[M,N] = A[M,K] . B[N,K]^T   (both operands K-contiguous, fp32
// accumulate) -- the o, gate/up, down and lm_head forwards of
// /root/reference/src/models/gpt.py:239, :278-281, :447.
//
// Why this shape (round 6).  In the two-chain training window a forward GEMM of one chain
// runs beside the other chain's kernels.  The persistent k_gemm_bf16 (gemm_bf16.hip) is as
// fast as hipBLASLt alone on o / down, but it keeps its 256 CUs for the whole launch, and
// in the step the other chain's memory-bound kernels beside it took 1.6-2x longer
// (norms 54 -> 89 us, cross-entropy 397 -> 755 us; the step -4.6 %, profiles/r6_gemm_fwd.md).
// The library kernel hands its CU back after every tile.  Here every workgroup computes
// ONE tile and ends, so the dispatcher hands CUs to the other stream tile by tile:
//   * tile 256 x BN, 2 x (BN / 64) waves, each 128 x 64 outputs = 8 x 4 tiles of
//     v_mfma_f32_16x16x32_bf16 (128 accumulator registers, <= 256 VGPRs: two waves per
//     SIMD); 12 ds_read_b128 per 32 MFMAs.  BN = 256 (8 waves, one workgroup per CU: the
//     wide projections, 128 FLOP per staged byte) or BN = 128 (4 waves, two workgroups per
//     CU: the N = 768 projections, whose 256-wide tiles would leave a quarter of the CUs
//     idle -- 192 tiles);
//   * BK = 32 stages by LDS-DMA (global_load_lds_dwordx4 from inline asm: SGPR base + 32-bit
//     lane offsets), a ring of NS (BN = 256: 4 x 32 KiB, three stages in flight; BN = 128:
//     3 x 24 KiB per workgroup): one counted vmcnt + one barrier per stage, placed between
//     the two MFMA halves of a k-step so the next stage's fragment reads overlap the second
//     half; the stage NS ahead is issued right after the barrier;
//   * LDS image rows of 64 bytes (4 chunks of 8 elements), chunk c of row r stored at
//     c ^ (2 * ((r >> 3) & 1)) -- the 16 rows x 4 chunks of a fragment read cover all 64
//     banks in every 16-lane group of ds_read_b128 (conflict-free); the swizzle is applied
//     to the DMA source address (the LDS side of an LDS-DMA is lane-linear);
//   * swapped product D = B_tile . A_tile^T, so a lane holds 4 consecutive columns of one
//     row per 16 x 16 tile; the epilogue stages the 256 x BN tile in the ring's LDS and
//     stores whole rows with 16-byte stores (write-through sc1 with flags & 1);
//   * XCD row bands: block b runs on the XCD of b % 8 (round-robin dispatch, speed only);
//     that XCD owns tile rows [x R, (x + 1) R), R = M / 2048, walked column by column, so
//     its A panels stay in its L2 and each B panel is fetched once per XCD.
//
// Requirements (launcher-checked): M % 256 == 0, N % 128 == 0, K % 32 == 0, 16-byte
// aligned rows (BN = 256 with N % 256 == 128, the lm_head: the last column tile clamps
// its B rows and masks its stores).  HK: operand / output format, 0 = bf16, 1 = IEEE half.
#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int FW_BM = 256, FW_BK = 32;

template <int BN>
struct FwCfg {
  static constexpr int WN = BN / 64;              // waves along N (2 along M)
  static constexpr int NW = 2 * WN;               // waves
  static constexpr int NS = BN == 256 ? 4 : 3;    // ring stages
  static constexpr int IMG_A = FW_BM * FW_BK;     // elements
  static constexpr int IMG_B = BN * FW_BK;
  static constexpr int STAGE = IMG_A + IMG_B;
  static constexpr int PA = 16 / NW;              // A pieces (16 rows) per wave per stage
  static constexpr int PB = (BN / 16) / NW;       // B pieces per wave per stage (2)
  static constexpr int P = PA + PB;               // DMA instructions per wave per stage
  static constexpr int CROW = BN + 8;             // epilogue staging row (elements; 16-byte pad)
  static constexpr int LDS = NS * STAGE > FW_BM * CROW ? NS * STAGE : FW_BM * CROW;
};

// byte offset of 16-byte chunk c (k = 8c .. 8c + 7) of image row r
__device__ __forceinline__ uint32_t fw_off(int r, int c) { return (uint32_t)(r * 64 + ((c ^ (((r >> 3) & 1) << 1)) << 4)); }

// one LDS-DMA piece: 64 lanes x 16 B -> 1 KiB at LDS byte address lds (wave-uniform)
__device__ __forceinline__ void fw_dma(const void* gbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(gbase), "s"(lds)
               : "memory", "m0");
}

// wait until at most n of this wave's vector-memory operations are outstanding (n is one of
// the counts the schedule produces); lgkmcnt(0) too: this wave's fragment reads are done
__device__ __forceinline__ void fw_wait(int n) {
  if (n >= 12) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

typedef __bf16 fw_bf16x4_t __attribute__((ext_vector_type(4)));
typedef _Float16 fw_f16x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t fw_u32x4_t __attribute__((ext_vector_type(4)));
template <int HK>
__device__ __forceinline__ uint2 fw_pack(const floatx4_t& v) {
  if constexpr (HK == 0) return __builtin_bit_cast(uint2, __builtin_convertvector(v, fw_bf16x4_t));
  else return __builtin_bit_cast(uint2, __builtin_convertvector(v, fw_f16x4_t));
}

}  // namespace

template <int HK, int BN>
__global__ __launch_bounds__(128 * (BN / 64), BN == 128 ? 2 : 1) void k_gemm_fwd(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, bf16_t* __restrict__ C, int M, int N, int K, int lda,
    int ldb, int ldc, int flags) {
  using Cf = FwCfg<BN>;
  __shared__ __attribute__((aligned(16))) bf16_t lds[Cf::LDS];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid & 1, wn = wid >> 1;
  const int l16 = lane & 15, lq = lane >> 4;

  // tile: XCD row bands (see the header), else row-major
  const int ntm = M / FW_BM, ntn = (N + BN - 1) / BN;
  const int bid = blockIdx.x;
  int tm, tn;
  if ((ntm & 7) == 0 && !(flags & 2)) {
    const int R = ntm >> 3, x = bid & 7, j = bid >> 3;
    tm = x * R + j % R;
    tn = j / R;
  } else {
    tm = bid / ntn;
    tn = bid - tm * ntn;
  }
  const int m0 = tm * FW_BM, n0 = tn * BN;

  // per-lane DMA byte offsets: wave w stages A rows (256 / NW) w + 16 j (PA pieces of 16
  // rows) and B rows 32 w + 16 j (PB pieces); lane i -> row + i / 4, physical chunk i % 4.
  // B rows past N (a ragged last column tile) re-read row N - 1: their columns are not stored.
  uint32_t aoff[Cf::PA], boff[Cf::PB];
#pragma unroll
  for (int j = 0; j < Cf::PA; ++j) {
    const int row = (FW_BM / Cf::NW) * wid + 16 * j + (lane >> 2);
    const int c = (lane & 3) ^ (((row >> 3) & 1) << 1);
    aoff[j] = (uint32_t)(row * lda + c * 8) * 2u;
  }
#pragma unroll
  for (int j = 0; j < Cf::PB; ++j) {
    const int row = (BN / Cf::NW) * wid + 16 * j + (lane >> 2);
    const int c = (lane & 3) ^ (((row >> 3) & 1) << 1);
    boff[j] = (uint32_t)((min(n0 + row, N - 1) - n0) * ldb + c * 8) * 2u;
  }
  const bf16_t* Ab = A + (size_t)m0 * lda;
  const bf16_t* Bb = B + (size_t)n0 * ldb;
  const uint32_t lbase = (uint32_t)(uintptr_t)lds;
  auto stage = [&](int s) {
    const uint32_t la = lbase + (uint32_t)((s % Cf::NS) * Cf::STAGE * 2);
    const uint32_t lb = la + Cf::IMG_A * 2;
    const bf16_t* ga = Ab + s * FW_BK;
    const bf16_t* gb = Bb + s * FW_BK;
#pragma unroll
    for (int j = 0; j < Cf::PA; ++j)
      fw_dma(ga, aoff[j], __builtin_amdgcn_readfirstlane(la + ((FW_BM / Cf::NW) * wid + 16 * j) * 64));
#pragma unroll
    for (int j = 0; j < Cf::PB; ++j)
      fw_dma(gb, boff[j], __builtin_amdgcn_readfirstlane(lb + ((BN / Cf::NW) * wid + 16 * j) * 64));
  };

  floatx4_t acc[4][8];  // [n-tile][m-tile]: D = B_tile . A_tile^T
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};

  // k-step s (one stage) runs its MFMAs from fragments read during k-step s - 1: the
  // first half (m-tiles 0-3), then [wait for stage s + 1, barrier, DMA of stage s + NS into
  // stage s's buffer -- every wave read it before this barrier --, fragment reads of stage
  // s + 1], then the second half, which covers the read latency.  Fragment registers
  // alternate between two sets (the loop is unrolled by two).
  const int ns = K / FW_BK;
  const char* const lc = reinterpret_cast<const char*>(lds);
  const uint32_t ra = fw_off(wm * 128 + l16, lq);  // (+ m-tile * 1 KiB)
  const uint32_t rb = fw_off(wn * 64 + l16, lq);   // (+ n-tile * 1 KiB)
  auto read_frags = [&](int s, bf16x8_t (&fa)[8], bf16x8_t (&fb)[4]) {
    const char* la = lc + (s % Cf::NS) * Cf::STAGE * 2;
    const char* lb = la + Cf::IMG_A * 2;
#pragma unroll
    for (int n = 0; n < 4; ++n) fb[n] = *reinterpret_cast<const bf16x8_t*>(lb + rb + n * 1024);
#pragma unroll
    for (int m = 0; m < 8; ++m) fa[m] = *reinterpret_cast<const bf16x8_t*>(la + ra + m * 1024);
  };
#pragma unroll
  for (int s = 0; s < Cf::NS; ++s)
    if (s < ns) stage(s);
  fw_wait(Cf::P * (min(Cf::NS, ns) - 1));  // stage 0 landed (the younger ones may fly)
  asm volatile("s_barrier" ::: "memory");
  bf16x8_t fa0[8], fb0[4], fa1[8], fb1[4];
  read_frags(0, fa0, fb0);
  auto kstep = [&](int s, bf16x8_t (&fa)[8], bf16x8_t (&fb)[4], bf16x8_t (&ga)[8], bf16x8_t (&gb)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n][m] = gw_mfma<HK>(fb[n], fa[m], acc[n][m]);
    __builtin_amdgcn_s_setprio(0);
    if (s + 1 < ns) {
      // stage s + 1 landed for this wave (stages s + 2 .. s + NS - 1 may be younger) and,
      // behind the barrier, for every wave; lgkmcnt(0) in the wait: this wave's reads of
      // stage s's buffer (issued a half k-step ago) are done before it is restaged
      fw_wait(Cf::P * min(Cf::NS - 2, ns - 2 - s));
      asm volatile("s_barrier" ::: "memory");
      if (s + Cf::NS < ns) stage(s + Cf::NS);
      read_frags(s + 1, ga, gb);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 4; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n][m] = gw_mfma<HK>(fb[n], fa[m], acc[n][m]);
    __builtin_amdgcn_s_setprio(0);
  };
#pragma unroll 1
  for (int s = 0; s < ns; s += 2) {
    kstep(s, fa0, fb0, fa1, fb1);
    if (s + 1 < ns) kstep(s + 1, fa1, fb1, fa0, fb0);
  }

  // epilogue: every wave is done with the ring (its last reads fed its last MFMAs), so
  // the tile is staged over it: lane holds C[wm*128 + 16m + l16][wn*64 + 16n + 4lq + 0..3]
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
      *reinterpret_cast<uint2*>(lds + (wm * 128 + 16 * m + l16) * Cf::CROW + wn * 64 + 16 * n + 4 * lq) =
          fw_pack<HK>(acc[n][m]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");
  // 256 rows x 2 BN bytes: thread t stores 16-byte chunk t % (BN / 8) of rows
  // t / (BN / 8) + 16 i (16 rows per instruction over the workgroup)
  constexpr int CPR = BN / 8;
  const int ch = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  const bool col_ok = n0 + ch * 8 < N;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(C + (size_t)m0 * ldc, 0, FW_BM * ldc * 2, 0x00020000);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = 16 * i + r0;
    const fw_u32x4_t v = *reinterpret_cast<const fw_u32x4_t*>(lds + row * Cf::CROW + ch * 8);
    const int off = (row * ldc + n0 + ch * 8) * 2;
    if (col_ok) {
      if (flags & 1)  // sc1: write-through (the C lines leave the XCD's L2)
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
    }
  }
}

// flags: 1 = write-through C stores, 2 = row-major tile order (A/B knob); bn: 128 or 256
// (0: 256 when the 256-wide tiles fill the CUs, else 128)
DLT_API int dlt_gemm_fwd(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb, int ldc,
                         int flags, int bn, int hk, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || M % FW_BM || N % 128 || K % FW_BK || lda % 8 || ldb % 8 || ldc % 8 || lda < K ||
      ldb < K || ldc < N)
    return -1;
  if (bn == 0) bn = (long)(M / FW_BM) * ((N + 255) / 256) >= 512 ? 256 : 128;
  if (bn != 128 && bn != 256) return -1;
  const long tiles = (long)(M / FW_BM) * ((N + bn - 1) / bn);
  if (tiles > 0x7fffffff || (long)FW_BM * ldc * 2 > 0x7fffffffL || (long)FW_BM * lda * 2 > 0xffffffffL ||
      (long)bn * ldb * 2 > 0xffffffffL)
    return -1;
  if (bn == 256)
    DLT_HK_DISPATCH(hk, k_gemm_fwd<HKC, 256><<<(int)tiles, 512, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, flags));
  else
    DLT_HK_DISPATCH(hk, k_gemm_fwd<HKC, 128><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, flags));
  DLT_CHECK_LAUNCH();
}
