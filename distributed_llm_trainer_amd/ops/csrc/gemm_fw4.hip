// Forward projection GEMM, 4-wave 256 x 256 tile, one tile per workgroup (gfx950 / MI355X):
//   C[M,N] = A[M,K] . B[N,K]^T   (both operands K-contiguous, fp32 accumulate)
// -- the o, gate/up, down and lm_head forwards of /root/reference/src/models/gpt.py:239,
// :278-281, :447.
//
// Why this shape (round 6).  In the two-chain training window a forward GEMM runs beside
// the other chain's memory-bound kernels; a persistent grid starves them (profiles/
// r6_gemm_fwd.md), so this kernel computes ONE tile per workgroup and hands its CU back
// to the dispatcher after every tile, like hipBLASLt's MT256x256x64 kernel it replaces.
//   * 256 threads = 4 waves (one per SIMD), each owning a 128 x 128 block of the tile:
//     8 x 8 accumulators of v_mfma_f32_16x16x32_bf16 = all 256 AGPRs (the MFMAs are
//     issued from inline asm with "+a" accumulators: the compiler's own MFMA selection
//     splits 256 loop-carried accumulators over both register halves and copies them
//     through v_accvgpr_read/write every iteration); 0.25 ds_read_b128 per MFMA;
//   * BK = 64 stages (128-byte operand rows: every LDS-DMA piece moves 8 whole 128-byte
//     lines), fragments of a stage read in two 32-deep halves; every instruction of the
//     loop is inline asm in a fixed order (MFMAs, fragment reads, DMA pieces, counted
//     vmcnt / lgkmcnt waits, barriers);
//   * schedules (launch flags): SCHED 1 (16) two 64 KiB stage buffers, the 3-phase form:
//     half 0 reads half 1's fragments; barrier; half 1 issues stage s + 2's DMA, waits
//     (vmcnt(16)) for stage s + 1, barrier, reads its half-0 fragments.  SCHED 3 (128) /
//     SCHED 5 (144): a ring of five 32 KiB image slots (A of stage s in slot 2s % 5, B in
//     2s + 1): stage s + 2's A image goes into the slot stage s - 1's B freed, so its DMA
//     spreads over half 0 and only the B image waits for the mid barrier; per-group
//     counted lgkmcnt waits.  SCHED 4 (default) / 5 use the INTERLEAVED epilogue below;
//     SCHED 1 / 3 stage the tile through LDS (swapped product, chunk-swizzled rows);
//   * interleaved epilogue (SCHED 4 / 5): n-tile u of a wave holds the B rows (output
//     columns) 8 v + u, v = 0..15, so register r of the 8 n-tiles is 8 consecutive columns
//     of row 16 t + 4 (l >> 4) + r: one 16-byte store per (m-tile, r) straight from the
//     accumulators, the 16 lanes of a row writing 256 contiguous bytes -- no LDS, no
//     barrier.  SCHED 4 pads the B pieces to 1040 bytes (conflict-free reads), SCHED 5
//     keeps the ring's 32 KiB slots (two-way bank conflicts on the B reads);
//   * SwiGLU epilogue (flags 1024, SCHED 4 / 5): the gate/up projection with
//     s = silu(gate) * up computed from the accumulators -- each wave's 128 B rows are 64
//     gate rows and the 64 up rows of the same intermediate indices, a row_ror:8 DPP move
//     pairs them in one lane, k_swiglu_fwd's arithmetic (same bits); gu keeps [gate | up];
//   * LDS images: A rows of 128 bytes, 16-byte chunk c of row r at c ^ (r & 7) (a 16-lane
//     group of ds_read_b128 covers all 64 banks); the DMA is lane-linear on the LDS side,
//     so every swizzle lives in the per-lane source offsets;
//   * tile order: XCD row bands (block b runs on the XCD of b % 8 under round-robin
//     dispatch; speed only): that XCD owns a band of tile rows and walks it column by
//     column (A panels stay in its L2); 2048: half-height bands, two per XCD; 2: row-major
//     (with N / 256 % 8 == 0 each XCD keeps a fixed set of B panels).  C stores: plain,
//     1 = write-through (sc1), 4 = nt.
//
// Requirements (launcher-checked): M % 256 == 0, N % 128 == 0, K % 64 == 0, K >= 128, rows
// 16-byte aligned; a ragged last column tile (N % 256 == 128, the lm_head) clamps its B
// rows and masks its stores.  HK: operand / output format, 0 = bf16, 1 = IEEE half.
#include "common.h"

#include <type_traits>
#include <utility>

namespace {

constexpr int F4_BM = 256, F4_BN = 256, F4_BK = 64;
constexpr int F4_IMG = 256 * F4_BK * 2;  // bytes of one operand image (32 KiB)
constexpr int F4_BUF = 2 * F4_IMG;       // A image then B image (64 KiB)
// SCHED 4's B image: 32 pieces of 8 rows x 128 B, each padded to 1040 B (see the header)
constexpr int F4_PIECE_BP = 1040;
constexpr int F4_IMG_BP = 32 * F4_PIECE_BP;
// SCHED 4's B swizzle: logical chunk c of a row of piece v (mod 16) sits at c ^ f4_fb(v)
__device__ __forceinline__ int f4_fb(int v) { return ((v + 4) >> 3) & 1; }

template <typename F, int... Is>
__device__ __forceinline__ void f4_sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
// compile-time loop: f(integral_constant<int, i>) for i = 0 .. N-1
template <int N, typename F>
__device__ __forceinline__ void f4_sfor(F&& f) {
  f4_sfor_impl(f, std::make_integer_sequence<int, N>{});
}

template <int HK>
__device__ __forceinline__ void f4_mfma(floatx4_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  if constexpr (HK == 0)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int OFF>
__device__ __forceinline__ void f4_read(bf16x8_t& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%c2" : "=v"(dst) : "v"(addr), "i"(OFF));
}

// LDS-DMA of one 1 KiB piece (64 lanes x 16 B, lane-linear at the wave-uniform LDS byte
// address lds) from SGPR base gbase + per-lane byte offset voff
__device__ __forceinline__ void f4_dma(const void* gbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(gbase), "s"(lds)
               : "memory");
}

typedef __bf16 f4_bf16x4_t __attribute__((ext_vector_type(4)));
typedef _Float16 f4_f16x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t f4_u32x4_t __attribute__((ext_vector_type(4)));
template <int HK>
__device__ __forceinline__ uint2 f4_pack(const floatx4_t& v) {
  if constexpr (HK == 0) return __builtin_bit_cast(uint2, __builtin_convertvector(v, f4_bf16x4_t));
  else return __builtin_bit_cast(uint2, __builtin_convertvector(v, f4_f16x4_t));
}

struct F4Frags {
  bf16x8_t a[8], b[8];  // m-tiles / n-tiles of one 32-deep stage
};

}  // namespace

template <int HK, int SCHED>
__global__ __launch_bounds__(256, 1) void k_gemm_fw4(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                     bf16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                     int ldc, int flags, bf16_t* __restrict__ S, int ldS,
                                                     unsigned long long* __restrict__ stamps) {
  // diagnostic (stamps != nullptr, tools/bench_gemm_fwd.py --stamps): wave 0 records
  // s_memrealtime (100 MHz) / s_memtime at start, after the prologue, after the main loop
  // and after its stores landed, plus the hardware ids, into stamps[16 * blockIdx.x ..]
  unsigned long long st_r[4], st_c[4];
  const bool stamp = stamps != nullptr && threadIdx.x < 64;
  if (stamp) { st_r[0] = __builtin_amdgcn_s_memrealtime(); st_c[0] = __builtin_amdgcn_s_memtime(); }
  // EPI: interleaved B n-tiles + direct epilogue (SCHED 4: padded B pieces, conflict-free;
  // SCHED 5: the five-slot ring, unpadded B with two-way bank conflicts on its reads)
  constexpr bool EPI = SCHED == 4 || SCHED == 5, PAD = SCHED == 4, RING = SCHED == 3 || SCHED == 5;
  constexpr int STG = PAD ? F4_IMG + F4_IMG_BP : F4_BUF;  // bytes of one stage buffer (2-buffer schedules)
  __shared__ __attribute__((aligned(16))) char lds[RING ? 5 * F4_IMG : 2 * STG];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid & 1, wn = wid >> 1;

  // tile: XCD row bands (see the header), else row-major
  const int ntm = M / F4_BM, ntn = (N + F4_BN - 1) / F4_BN;
  const int bid = blockIdx.x;
  int tm, tn;
  if ((ntm & 15) == 0 && (flags & 2048)) {
    // 2048: half-height bands, two per XCD (band x, then band x + 8): R = ntm / 16 rows
    const int R = ntm >> 4, x = bid & 7, j = bid >> 3, per = R * ntn;
    const int band = j < per ? x : x + 8, jj = j < per ? j : j - per;
    tm = band * R + jj % R;
    tn = jj / R;
  } else if ((ntm & 7) == 0 && !(flags & 2)) {
    const int R = ntm >> 3, x = bid & 7, j = bid >> 3;
    tm = x * R + j % R;
    tn = j / R;
  } else {
    tm = bid / ntn;
    tn = bid - tm * ntn;
  }
  const int m0 = tm * F4_BM, n0 = tn * F4_BN;

  // DMA piece j (0..7) of wave w: rows 64 w + 8 j + i / 8 of an operand image, lane i ->
  // physical chunk i % 8 = logical chunk (i % 8) ^ (i / 8).  B rows past N re-read row
  // N - 1 (their columns are not stored).
  const int lr = lane >> 3, lc = (lane & 7) ^ lr;
  uint32_t aoff[8], boff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 64 * wid + 8 * j + lr;
    aoff[j] = (uint32_t)(row * lda + lc * 8) * 2u;
    // SCHED 4: piece 8 w + j of the B image holds rows 8 v + u (v = piece % 16) of n-tile u
    // (SCHED 5: logical chunk c of B-image row 8 v + u at c ^ (v & 7))
    const int blc = PAD ? (lane & 7) ^ f4_fb((8 * wid + j) & 15) : EPI ? (lane & 7) ^ ((8 * wid + j) & 7) : lc;
    // SWIGLU (flags & 1024, EPI schedules): the tile covers intermediate indices
    // [128 tn, 128 tn + 128); wave-half wn of its B rows = 64 gate rows then the 64 up rows
    // of indices 128 tn + 64 wn + 0..63 (Wgu rows j and I + j)
    const int brow = (flags & 1024) ? ((row & 127) >> 6) * (N >> 1) + 64 * (row >> 7) + (row & 63)
                                    : min(n0 + row, N - 1) - n0;
    boff[j] = (uint32_t)(brow * ldb + blc * 8) * 2u;
  }
  const bf16_t* Ab = A + (size_t)m0 * lda;
  const bf16_t* Bb = B + (size_t)((flags & 1024) ? 128 * tn : n0) * ldb;
  const uint32_t lbase = (uint32_t)(uintptr_t)lds;
  // LDS byte offsets of stage s's A and B images: SCHED 0 / 1 two 64 KiB stage buffers;
  // SCHED 2 a ring of five 32 KiB image slots, A of stage s in slot 2s % 5, B in (2s + 1) % 5
  auto slot_a = [&](int s) -> uint32_t {
    if constexpr (RING) return (uint32_t)(((2 * s) % 5) * F4_IMG);
    else return (uint32_t)((s & 1) * STG);
  };
  auto slot_b = [&](int s) -> uint32_t {
    if constexpr (RING) return (uint32_t)(((2 * s + 1) % 5) * F4_IMG);
    else return (uint32_t)((s & 1) * STG + F4_IMG);
  };
  // piece p of stage s: A pieces 0..7, B pieces 8..15
  auto piece = [&](int s, int p) {
    if (p < 8)
      f4_dma(Ab + s * F4_BK, aoff[p], __builtin_amdgcn_readfirstlane(lbase + slot_a(s) + (64 * wid + 8 * p) * 128));
    else
      f4_dma(Bb + s * F4_BK, boff[p - 8],
             __builtin_amdgcn_readfirstlane(lbase + slot_b(s) +
                                            (PAD ? (8 * wid + p - 8) * F4_PIECE_BP : (64 * wid + 8 * (p - 8)) * 128)));
  };

  floatx4_t acc[8][8];  // [n-tile u][m-tile t]: D = B_tile . A_tile^T
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = floatx4_t{0.f, 0.f, 0.f, 0.f};

  // fragment of 16 rows x 32 k (half h of a stage): lane l reads row base + (l & 15),
  // logical chunk 4 h + (l >> 4) at physical chunk (4 h + (l >> 4)) ^ (l & 7)
  const uint32_t loff = (uint32_t)((lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) << 4));
  const uint32_t fa_base = lbase + (uint32_t)(wm * 128 * 128);
  // SCHED 4 n-tile u: rows 8 v + u of pieces wn * 16 + v (v = l & 15), chunk (4 h + q) ^ fb(v)
  const uint32_t fb_base =
      PAD   ? lbase + (uint32_t)((wn * 16 + (lane & 15)) * F4_PIECE_BP + (((lane >> 4) ^ f4_fb(lane & 15)) << 4))
      : EPI ? (uint32_t)((wn * 128 + 8 * (lane & 15)) * 128 + (((lane >> 4) ^ (lane & 7)) << 4))  // + lbase at use
            : lbase + (uint32_t)(wn * 128 * 128);
  // read slot r (0..15) of half h of stage s: slots 0..7 the n-tiles, 8..15 the m-tiles
  auto read_slot = [&](auto r_c, int s, int h, F4Frags& f) {
    constexpr int r = decltype(r_c)::value;
    const uint32_t o = loff ^ (uint32_t)(64 * h);
    if constexpr (r < 8) {
      if constexpr (PAD) f4_read<r * 128>(f.b[r], fb_base + slot_b(s) + (uint32_t)(64 * h));
      else if constexpr (EPI) f4_read<r * 128>(f.b[r], lbase + (fb_base ^ (uint32_t)(64 * h)) + slot_b(s));
      else f4_read<r * 2048>(f.b[r], fb_base + slot_b(s) + o);
    } else {
      f4_read<(r - 8) * 2048>(f.a[r - 8], fa_base + slot_a(s) + o);
    }
  };
  auto mfma_group = [&](auto g_c, F4Frags& f) {
    constexpr int g = decltype(g_c)::value;
    f4_sfor<8>([&](auto u_c) {
      constexpr int u = decltype(u_c)::value;
      if constexpr (EPI) f4_mfma<HK>(acc[u][g], f.a[g], f.b[u]);
      else f4_mfma<HK>(acc[u][g], f.b[u], f.a[g]);
    });
  };

  // one stage (64 deep): half 0 = 64 MFMAs on f0 (its k 0..31) with half 1's 16 fragment
  // reads interleaved; then (NEXT) wait for stage s + 1 (this wave's only DMAs in flight)
  // and for this wave's reads, barrier (every wave is done with stage s's buffer), half 1
  // = 64 MFMAs on f1 with (DMA) stage s + 2's 16 pieces into stage s's buffer and (NEXT)
  // stage s + 1's half-0 reads interleaved, two of each per 8-MFMA group
  F4Frags f0, f1;
  // 64 MFMAs of one half on f with hook(i) after MFMA i (i = 8 t + u)
  auto half = [&](F4Frags& f, auto&& hook) {
    f4_sfor<64>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      if constexpr (EPI) f4_mfma<HK>(acc[i & 7][i >> 3], f.a[i >> 3], f.b[i & 7]);
      else f4_mfma<HK>(acc[i & 7][i >> 3], f.b[i & 7], f.a[i >> 3]);
      hook(i_c);
    });
  };
  // one stage (64 deep), SCHED 0: half 0 = 64 MFMAs on f0 (its k 0..31) with half 1's 16
  // fragment reads interleaved; then (NEXT) wait for stage s + 1 (this wave's only DMAs in
  // flight) and this wave's reads, barrier (every wave is done with stage s's buffer);
  // half 1 = 64 MFMAs on f1 with (DMA) stage s + 2's 16 pieces into stage s's buffer and
  // (NEXT) stage s + 1's half-0 reads interleaved, two of each per 8-MFMA group.
  // SCHED 1 (the 3-phase form): half 0 reads f1 over its first 48 MFMAs; barrier; half 1
  // issues stage s + 2's pieces over its first 48 MFMAs, then waits for stage s + 1 only
  // (vmcnt(16): the new pieces may fly), barrier, and reads stage s + 1's half-0 fragments
  // one per MFMA over its last 16 -- stage s + 1 has a whole stage of DMA latency cover.
  // SCHED 2 (five 32 KiB image slots): as SCHED 1, but stage s + 2's A image goes into the
  // slot stage s - 1's B image freed, so its 8 pieces spread over half 0 (one per 8 MFMAs)
  // and only the B pieces (into stage s's A slot) wait for the mid barrier: the 16 DMA
  // issues per stage no longer crowd one half.
  auto stage = [&](int s, auto next_c, auto dma_c) {
    constexpr bool NEXT = decltype(next_c)::value, DMA = decltype(dma_c)::value;
    if constexpr (RING) {
      // SCHED 3: the barrier at MFMA 39 of half 1 and stage s + 1's reads over MFMAs 40..55
      // (8 MFMAs of cover before the stage ends); the next half 0 waits per 8-MFMA group
      // for exactly the fragments it uses (n-tiles first, then m-tile t before group t)
      constexpr int BAR = 39;
      half(f0, [&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        if constexpr (i % 8 == 7 && i < 63) {
          // before group t = (i + 1) / 8: reads 0 .. 8 + t of f0 done; younger: the rest of
          // f0's (7 - t) and the f1 reads issued so far (one per 3 MFMAs, i % 3 == 2)
          constexpr int t = (i + 1) / 8;
          constexpr int nf1 = (i + 1) / 3 < 16 ? (i + 1) / 3 : 16;
          constexpr int X = (7 - t) + nf1 > 15 ? 15 : (7 - t) + nf1;
          asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(X) : "memory");
        }
        if constexpr (DMA && i % 8 == 7) piece(s + 2, i / 8);
        if constexpr (i % 3 == 2 && i / 3 < 16) read_slot(std::integral_constant<int, i / 3>{}, s, 1, f1);
      });
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      half(f1, [&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        if constexpr (DMA && i % 5 == 0 && i / 5 < 8) piece(s + 2, 8 + i / 5);
        if constexpr (NEXT && i == BAR) {
          if constexpr (DMA) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if constexpr (NEXT && i > BAR && i <= BAR + 16) read_slot(std::integral_constant<int, i - BAR - 1>{}, s + 1, 0, f0);
      });
      if constexpr (NEXT) {
        // the next half 0's group 0 needs reads 0..8 (8 n-tiles + m-tile 0)
        asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
        return;
      }
    } else {
      half(f0, [&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        if constexpr (i % 3 == 2 && i / 3 < 16) read_slot(std::integral_constant<int, i / 3>{}, s, 1, f1);
      });
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      half(f1, [&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        if constexpr (DMA && i % 3 == 0 && i / 3 < 16) piece(s + 2, i / 3);
        if constexpr (NEXT && i == 47) {
          if constexpr (DMA) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if constexpr (NEXT && i >= 48) read_slot(std::integral_constant<int, i - 48>{}, s + 1, 0, f0);
      });
    }
    // the next stage's first MFMAs read f0: this wave's half-0 reads must have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  const int ns = K / F4_BK;  // >= 2 (launcher-checked)
  // prologue: stages 0 and 1 in flight, stage 0 landed, its half-0 fragments read
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int p = 0; p < 16; ++p) piece(s, p);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  f4_sfor<16>([&](auto r_c) { read_slot(r_c, 0, 0, f0); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (stamp) { st_r[1] = __builtin_amdgcn_s_memrealtime(); st_c[1] = __builtin_amdgcn_s_memtime(); }

  using T_ = std::true_type;
  using F_ = std::false_type;
  int s = 0;
#pragma unroll 1
  for (; s + 2 < ns; ++s) stage(s, T_{}, T_{});
  stage(s, T_{}, F_{});
  stage(s + 1, F_{}, F_{});
  if (stamp) { st_r[2] = __builtin_amdgcn_s_memrealtime(); st_c[2] = __builtin_amdgcn_s_memtime(); }

  // epilogue: 16 wait states for the last MFMAs' accumulators
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const int l16 = lane & 15, q = lane >> 4;
  if constexpr (EPI) {
    // SCHED 4 (product D = A_tile . B_tile^T): lane l, register r of tile (u, t) is output
    // row 16 t + 4 (l >> 4) + r, column wn*128 + 8 (l & 15) + u (n-tile u holds columns
    // 8 v + u), so the eight n-tiles give 8 consecutive columns and the 16 lanes of a row
    // 256 contiguous bytes: one 16-byte store per (m-tile, r), 4 rows per instruction, no LDS
    const int col = n0 + wn * 128 + 8 * l16;
    const bool col_ok = n0 + wn * 128 < N;
    const auto rs =
        __builtin_amdgcn_make_buffer_rsrc(C + (size_t)(m0 + wm * 128) * ldc, 0, 128 * ldc * 2, 0x00020000);
    if (flags & 1024) {
      // SWIGLU: lanes v = l & 15 < 8 hold gate indices jb + 8 v + u, lanes v + 8 the up values
      // of the same indices; after a row_ror:8 exchange each lane of the pair has both and
      // computes s = silu(g) * u -- k_swiglu_fwd's arithmetic on the bf16-rounded g and u,
      // same bits -- for 4 of the 8 indices.  gu keeps its [M, 2I] layout (gate | up).
      const int I = N >> 1, jb = 128 * tn + 64 * wn, v = l16;
      const int gcol = (v < 8 ? jb : I + jb) + 8 * (v & 7), e0 = v < 8 ? 0 : 4;
      const auto rss =
          __builtin_amdgcn_make_buffer_rsrc(S + (size_t)(m0 + wm * 128) * ldS, 0, 128 * ldS * 2, 0x00020000);
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          floatx4_t lo{acc[0][t][r], acc[1][t][r], acc[2][t][r], acc[3][t][r]};
          floatx4_t hi{acc[4][t][r], acc[5][t][r], acc[6][t][r], acc[7][t][r]};
          const uint2 a = f4_pack<HK>(lo), b = f4_pack<HK>(hi);
          const f4_u32x4_t P{a.x, a.y, b.x, b.y};
          f4_u32x4_t Q;
#pragma unroll
          for (int d = 0; d < 4; ++d) Q[d] = (uint32_t)__builtin_amdgcn_mov_dpp((int)P[d], 0x128, 0xf, 0xf, false);
          const int row = 16 * t + 4 * q + r;
          const int off = (row * ldc + gcol) * 2;
          if (flags & 1) __builtin_amdgcn_raw_buffer_store_b128(P, rs, off, 0, 16);
          else if (flags & 4) __builtin_amdgcn_raw_buffer_store_b128(P, rs, off, 0, 2);
          else __builtin_amdgcn_raw_buffer_store_b128(P, rs, off, 0, 0);
          const f4_u32x4_t G = v < 8 ? P : Q, U = v < 8 ? Q : P;
          uint32_t o2[2];
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const int w0 = (e0 + e) >> 1;  // dword holding elements e0 + e, e0 + e + 1
            float sv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float gv = h2f<HK>((uint16_t)(G[w0] >> (16 * h)));
              const float uv = h2f<HK>((uint16_t)(U[w0] >> (16 * h)));
              sv[h] = gv * dlt_sigmoid(gv) * uv;
            }
            o2[e >> 1] = (uint32_t)f2h<HK>(sv[0]) | ((uint32_t)f2h<HK>(sv[1]) << 16);
          }
          const int soff = (row * ldS + jb + 8 * (v & 7) + e0) * 2;
          typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
          __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{o2[0], o2[1]}, rss, soff, 0, 0);
        }
    } else if (col_ok) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          floatx4_t lo{acc[0][t][r], acc[1][t][r], acc[2][t][r], acc[3][t][r]};
          floatx4_t hi{acc[4][t][r], acc[5][t][r], acc[6][t][r], acc[7][t][r]};
          const uint2 a = f4_pack<HK>(lo), b = f4_pack<HK>(hi);
          const f4_u32x4_t v{a.x, a.y, b.x, b.y};
          const int off = ((16 * t + 4 * q + r) * ldc + col) * 2;
          if (flags & 1) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);  // sc1 write-through
          else if (flags & 4) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 2);  // nt
          else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
        }
    }
  } else {
    // wave w stages its 128 x 128 block in bytes [32 KiB w, 32 KiB (w + 1)) once every wave
    // is done with the ring: row r (256 bytes), 16-byte chunk c at c ^ (r & 15)
    asm volatile("s_barrier" ::: "memory");
    char* const stg = lds + wid * 32768;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = 16 * t + l16, c = 2 * u + (q >> 1);
        *reinterpret_cast<uint2*>(stg + r * 256 + ((c ^ (r & 15)) << 4) + (q & 1) * 8) = f4_pack<HK>(acc[u][t]);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's own block only
    const int ch = lane & 15, r0 = lane >> 4;
    const int col = n0 + wn * 128 + ch * 8;
    const bool col_ok = col < N;
    const auto rs =
        __builtin_amdgcn_make_buffer_rsrc(C + (size_t)(m0 + wm * 128) * ldc, 0, 128 * ldc * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int r = 4 * i + r0;
      const f4_u32x4_t v = *reinterpret_cast<const f4_u32x4_t*>(stg + r * 256 + ((ch ^ (r & 15)) << 4));
      const int off = (r * ldc + col) * 2;
      if (col_ok) {
        if (flags & 1) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);  // sc1 write-through
        else if (flags & 4) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 2);  // nt
        else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
      }
    }
  }
  if (stamp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_r[3] = __builtin_amdgcn_s_memrealtime();
    st_c[3] = __builtin_amdgcn_s_memtime();
    unsigned long long* o = stamps + 16 * (size_t)blockIdx.x;
    if (lane < 4) {
      o[lane] = lane == 0 ? st_r[0] : lane == 1 ? st_r[1] : lane == 2 ? st_r[2] : st_r[3];
      o[4 + lane] = lane == 0 ? st_c[0] : lane == 1 ? st_c[1] : lane == 2 ? st_c[2] : st_c[3];
    }
    if (lane == 0) {
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      o[8] = hw;
      o[9] = xcc;
      o[10] = (unsigned long long)((tm << 16) | tn);
    }
  }
}

// flags: 1 = write-through (sc1) C stores, 4 = nt C stores, 2 = row-major tile order (A/B knob);
// schedule: 16 = SCHED 1, 128 = SCHED 3, 144 = SCHED 5, else SCHED 4; 1024 = SwiGLU epilogue (SCHED 4 / 5)
DLT_API int dlt_gemm_fw4(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb, int ldc,
                         int flags, int hk, bf16_t* S, int ldS, unsigned long long* stamps, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || M % F4_BM || N % 128 || K % F4_BK || K < 2 * F4_BK || lda % 8 || ldb % 8 ||
      ldc % 8 || lda < K || ldb < K || ldc < N)
    return -1;
  // SWIGLU epilogue (flags & 1024): N = 2I with I % 128 == 0, s [M, ldS >= I], EPI schedules
  const int sched_bits = flags & (16 | 128);  // 0: SCHED 4, 16 | 128: SCHED 5
  if ((flags & 1024) && (S == nullptr || N % 256 || ldS < N / 2 || ldS % 8 || sched_bits == 16 || sched_bits == 128 ||
                         128L * ldS * 2 > 0x7fffffffL || (long)(N / 2 + 127) * ldb * 2 > 0xffffffffL))
    return -1;
  const long tiles = (long)(M / F4_BM) * ((N + F4_BN - 1) / F4_BN);
  if (tiles > 0x7fffffff || 128L * ldc * 2 > 0x7fffffffL || 256L * lda * 2 > 0xffffffffL ||
      256L * ldb * 2 > 0xffffffffL)
    return -1;
  if ((flags & 128) && (flags & 16))
    DLT_HK_DISPATCH(hk, k_gemm_fw4<HKC, 5><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, flags, S, ldS, stamps));
  else if (flags & 128)
    DLT_HK_DISPATCH(hk, k_gemm_fw4<HKC, 3><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, flags, S, ldS, stamps));
  else if (flags & 16)
    DLT_HK_DISPATCH(hk, k_gemm_fw4<HKC, 1><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, flags, S, ldS, stamps));
  else
    DLT_HK_DISPATCH(hk, k_gemm_fw4<HKC, 4><<<(int)tiles, 256, 0, st>>>(A, B, C, M, N, K, lda, ldb, ldc, flags, S, ldS, stamps));
  DLT_CHECK_LAUNCH();
}
