// Weight-gradient GEMM for the deferred wgrads of the transformer block (gfx950 / MI355X):
//   dW[Nr, Nc] (fp32)  (+)=  dY[T, Nr]^T . X[T, Nc]        (bf16 in, fp32 accumulate)
// -- the weight gradients of the projections of /root/reference/src/models/gpt.py:185-187,239
// (q/k/v/o) and :278-281 (gate/up/down), reduced over the T = GA x B x S tokens of one
// gradient-accumulation window (models/engine.py defers them to one GEMM per weight).
//
// Both operands are TOKEN-major: the reduction index is the outer (row) index, so an MFMA
// fragment -- 8 consecutive tokens of one output row or column -- is a column of the
// row-major tile.  Tiles are staged row-major by LDS-DMA (whole 128/256-byte token rows,
// fully coalesced) and the fragments are read with ds_read_b64_tr_b16, the hardware
// transpose (cdna_hip_programming.md T10): two 4-token reads per 16x16x32 operand.
//
// Structure: the persistent projection GEMM's pipeline (gemm_bf16.hip) -- 256 (rows of dW)
// x 192 (columns) tiles, BK = 64 tokens, 512 threads = 8 waves as 4 (M) x 2 (N), each wave
// 64 x 96 = 4 x 6 tiles of v_mfma_f32_16x16x32_bf16, 4 quadrant phases per K-tile, one
// staging unit per phase (restaged >= 2 phases after its last read, retired by a counted
// vmcnt(4) one phase before it is read), waves 4-7 one barrier behind 0-3.  Staging units
// are separate row-major LDS images:
//   A0 / A1: the 32-column halves of every wave's 64 rows of dW   [64 tok][128] (256-B rows)
//   B0: n-tiles 0..3 of both N halves [64 tok][128];  B1: n-tiles 4..5 [64 tok][64] (128-B rows)
// Source-side XOR swizzle of the 16-byte chunks of a token row (pc = lc ^ 2v(t)) makes
// every transposed read conflict-free: a 32-lane half reads 8 token rows x 32 bytes, which
// land on 8 distinct 32-byte bank slots (v(t) distinct over those rows; for 128-byte
// rows the even / odd rows already sit in different bank halves).
//
// The reduction over T is split over workgroups (`splits`, chosen by the caller so that
// tiles x splits fills the 256 CUs): each split writes its fp32 partial tile and
// k_splitk_acc (elementwise.hip) adds the partials into dW in a FIXED order -- no float
// atomics, bitwise run-to-run reproducible (DDP replicas stay identical).  With one split
// the kernel adds straight into dW.
//
// Requirements (launcher-checked): Nr % 128 == 0 (a last half tile when Nr % 256 == 128),
// Nc % 192 == 0 (or Nc % 128 == 0: the 256 x 128 column-tile instance, BN = 128, for
// hidden sizes such as 1024), T % 128 == 0, 16-byte aligned rows.
//
// HK: operand format, 0 = bf16, 1 = IEEE half (--mixed_precision fp16).  Staging and the
// transposed reads move 16-bit words either way; only the MFMA differs
// (v_mfma_f32_16x16x32_f16, same shape and rate).
#include "common.h"

// shared token-major staging / transposed-read helpers (also used by the dgrad form of
// k_gemm_bf16, whose weight operand is reduction-major)
#include "gemm_common.h"

// One (256-row x 192-column dW tile, K-tile range) segment: prologue, the 8-phase main
// loop over K-tiles [kt0, kt0 + nk) (nk even >= 2), epilogue into dst (row stride ldd;
// accumulate: dst += acc, else dst = acc).  Ends with every wave past its last LDS read,
// so a workgroup may run segments back to back (stream-K).
// BN: dW tile columns, 192 (6 n-tiles per wave: B0 + B1) or 128 (4 per wave, B0 only; the
// 8-phase schedule's counted waits hold unchanged with an empty B1 unit -- every wait
// leaves exactly the next K-tile's A0 / B0 units in flight either way).
template <int HK, int BN = 192>
__device__ __forceinline__ void gw_segment(bf16_t* lds, const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                           int r0, int c0, int kt0, int nk, bool half_tile, int ldy, int ldx,
                                           float* __restrict__ dst, int ldd, bool accumulate) {
  static_assert(BN == 192 || BN == 128, "dW column tile of 192 or 128");
  constexpr int NT = BN / 32, NH = NT / 2;  // n-tiles per wave / per quadrant
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = wid >> 2;
  const int wm = wid & 3, wn = wid >> 2;
  const int l16 = lane & 15, lq = lane >> 4;

  // images of buffer b (element offsets into lds): A0, A1, B0, B1.  DMA destinations are
  // LDS pointers; the asm transposed reads take the 32-bit LDS address (the low word of
  // the generic address of a __shared__ object, as in attention.hip)
  auto eA = [&](int b, int q) { return b * GW_BUF + q * GW_IMG_A; };
  auto eB0 = [&](int b) { return b * GW_BUF + 2 * GW_IMG_A; };
  auto eB1 = [&](int b) { return b * GW_BUF + 3 * GW_IMG_A; };
  auto laddr = [&](int e) { return (uint32_t)(uintptr_t)(lds + e); };
  auto imgA = [&](int b, int q) { return laddr(eA(b, q)); };
  auto imgB0 = [&](int b) { return laddr(eB0(b)); };
  auto imgB1 = [&](int b) { return laddr(eB1(b)); };

  // per-lane source offsets (bytes from the K-tile's first token row at the tile's column
  // origin): 16 KB units = 16 DMA instructions (2 per wave, 4 token rows each), B1 = 8
  // (1 per wave, 8 rows each)
  uint32_t oa[2][2], ob0[2], ob1;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = (wid * 2 + j) * 64 + lane;  // chunk index in the image
    const int t = e >> 4, pc = e & 15;
    const int lc = pc ^ (2 * gw_v256(t));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int col = gw_amap(q, lc * 8);
      if (half_tile) col &= 127;
      oa[q][j] = (uint32_t)(t * ldy + col) * 2u;
    }
    ob0[j] = (uint32_t)(t * ldx + gw_b0map<BN>(lc * 8)) * 2u;
  }
  {
    const int e = wid * 64 + lane;
    const int t = e >> 3, pc = e & 7;
    const int lc = pc ^ (2 * gw_v128(t));
    ob1 = (uint32_t)(t * ldx + gw_b1map(lc * 8)) * 2u;
  }
  const bf16_t* const Ab = dY + (size_t)kt0 * GW_BK * ldy + r0;
  const bf16_t* const Bb = X + (size_t)kt0 * GW_BK * ldx + c0;
  auto stA = [&](int kt, int q, int b) {  // kt relative to kt0
    const char* g = (const char*)(Ab + (size_t)kt * GW_BK * ldy);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((gw_gbl_cvptr_t)(g + oa[q][j]),
                                       (gw_lds_vptr_t)(lds + eA(b, q) + (wid * 2 + j) * 512), 16, 0, 0);
  };
  auto stB0 = [&](int kt, int b) {
    const char* g = (const char*)(Bb + (size_t)kt * GW_BK * ldx);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((gw_gbl_cvptr_t)(g + ob0[j]),
                                       (gw_lds_vptr_t)(lds + eB0(b) + (wid * 2 + j) * 512), 16, 0, 0);
  };
  auto stB1 = [&](int kt, int b) {
    if constexpr (BN == 192) {
      const char* g = (const char*)(Bb + (size_t)kt * GW_BK * ldx);
      __builtin_amdgcn_global_load_lds((gw_gbl_cvptr_t)(g + ob1),
                                       (gw_lds_vptr_t)(lds + eB1(b) + wid * 512), 16, 0, 0);
    }
  };

  floatx4_t acc[NT][4];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t fa[2][2], fb0[NH][2], fb1[NH][2];

  GwLane<256> L256;
  GwLane<128> L128;
  L256.init(lane);
  L128.init(lane);
  // per-lane read bases: A fragments k = 2 wm + mt (16-column blocks of the A image), B0
  // k = 4 wn + nt, B1 k = 2 wn + j
  uint32_t ka[2], kb0[4], kb1[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ka[j] = L256.base + L256.koff(2 * wm + j);
    kb1[j] = L128.base + L128.koff(2 * wn + j);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) kb0[j] = L256.base + L256.koff(4 * wn + j);
  auto read_a = [&](int b, int qm) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[mt][s] = gw_frag<256>(imgA(b, qm) + ka[mt], s);
  };
  // BN 192: n-half 0: n-tiles 0..2 (B0); n-half 1: n-tile 3 (B0) and 4..5 (B1)
  // BN 128: n-half qn: n-tiles 2qn, 2qn + 1, both from B0
  auto read_b = [&](int b, int qn, bf16x8_t (&fb)[NH][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (BN == 128) {
#pragma unroll
        for (int nt = 0; nt < NH; ++nt) fb[nt][s] = gw_frag<256>(imgB0(b) + kb0[qn * NH + nt], s);
      } else if (qn == 0) {
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) fb[nt][s] = gw_frag<256>(imgB0(b) + kb0[nt], s);
      } else {
        fb[0][s] = gw_frag<256>(imgB0(b) + kb0[3], s);
        fb[1][s] = gw_frag<128>(imgB1(b) + kb1[0], s);
        fb[2][s] = gw_frag<128>(imgB1(b) + kb1[1], s);
      }
    }
  };
  // retire this wave's transposed reads (asm, invisible to the compiler's lgkmcnt
  // tracking: the fragments are in/out operands so no MFMA is scheduled above the wait)
  auto lds_wait = [&](bf16x8_t (&fb)[NH][2]) {
    if constexpr (NH == 3)
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                     "+v"(fb[1][0]), "+v"(fb[1][1]), "+v"(fb[2][0]), "+v"(fb[2][1])::"memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                     "+v"(fb[1][0]), "+v"(fb[1][1])::"memory");
  };
  auto mma = [&](int qm, int qn, bf16x8_t (&fb)[NH][2]) {
    lds_wait(fb);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[qn * NH + nt][qm * 2 + mt] = gw_mfma<HK>(fb[nt][s], fa[mt][s], acc[qn * NH + nt][qm * 2 + mt]);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: K-tile 0 complete in buffer 0, A0/B0 of K-tile 1 in flight
  stA(0, 0, 0);
  stB0(0, 0);
  stB1(0, 0);
  stA(0, 1, 0);
  stA(1, 0, 1);
  stB0(1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (half == 1) __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nk; kt += 2) {
    const bool more = kt + 2 < nk;
    // ---- phase 1: buffer 0, q0 ; B1 of K-tile kt+1
    read_b(0, 0, fb0);
    read_a(0, 0);
    stB1(kt + 1, 1);
    __builtin_amdgcn_s_barrier();
    mma(0, 0, fb0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: q1 ; A1 of kt+1
    read_b(0, 1, fb1);
    stA(kt + 1, 1, 1);
    __builtin_amdgcn_s_barrier();
    mma(0, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: q2 ; A0 of kt+2 into buffer 0
    read_a(0, 1);
    if (more) stA(kt + 2, 0, 0);
    __builtin_amdgcn_s_barrier();
    mma(1, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: q3 (registers) ; B0 of kt+2 ; retire kt+1
    if (more) {
      stB0(kt + 2, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    mma(1, 0, fb0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 5: buffer 1, q0 ; B1 of kt+2
    read_b(1, 0, fb0);
    read_a(1, 0);
    if (more) stB1(kt + 2, 0);
    __builtin_amdgcn_s_barrier();
    mma(0, 0, fb0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 6: q1 ; A1 of kt+2
    read_b(1, 1, fb1);
    if (more) stA(kt + 2, 1, 0);
    __builtin_amdgcn_s_barrier();
    mma(0, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 7: q2 ; A0 of kt+3 into buffer 1
    read_a(1, 1);
    if (more) stA(kt + 3, 0, 1);
    __builtin_amdgcn_s_barrier();
    mma(1, 1, fb1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 8: q3 ; B0 of kt+3 ; retire kt+2
    if (more) {
      stB0(kt + 3, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    mma(1, 0, fb0);
    __builtin_amdgcn_s_barrier();
  }
  if (half == 0) __builtin_amdgcn_s_barrier();

  // epilogue: acc[nt][mt] = D[n][m]: lane owns tile row wm*64 + mt*16 + l16 and the 4
  // consecutive columns wn*BN/2 + nt*16 + lq*4 .. +3 (one float4)
  if (half_tile && wm >= 2) return;  // rows past Nr (wave-uniform; no barrier follows in this segment)
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    float* row = dst + (size_t)(wm * 64 + mt * 16 + l16) * ldd + wn * (BN / 2) + lq * 4;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float4* p = reinterpret_cast<float4*>(row + nt * 16);
      float4 v = {acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]};
      if (accumulate) {
        const float4 o = *p;
        v.x += o.x;
        v.y += o.y;
        v.z += o.z;
        v.w += o.w;
      }
      *p = v;
    }
  }
}

template <int HK, int BN = 192>
__global__ __launch_bounds__(512, 1) void k_gemm_wgrad(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                                       float* __restrict__ out, int T, int Nr, int Nc, int ldy,
                                                       int ldx, int splits, int accumulate) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * GW_BUF];
  // workgroup -> (row tile, split, column tile), XCD-aware: the dispatcher deals workgroup
  // ids round-robin to the 8 XCDs, so ids i, i + 8, ... share an XCD's L2.  A unit u =
  // (row tile, split) reads one [T / splits, 256] slab of dY, which every column tile of
  // that row needs: the ntc column tiles of unit u are ids 8 * (ntc * (u / 8) + c) + u % 8,
  // all on XCD u % 8 and dispatched together, so the slab is fetched from HBM once, not
  // ntc times (the 3.3 GB dlogits slab of the lm_head gradient was read 4x before).
  // The grid is padded to whole groups of 8 units; padding workgroups exit at once.
  const int ntc = Nc / BN;
  const int nunits = ((Nr + 255) / 256) * splits;
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int u = (q / ntc) * 8 + xcd;
  if (u >= nunits) return;  // padding (uniform over the workgroup, before any barrier)
  const int split = u % splits;
  const int r0 = (u / splits) * 256, c0 = (q % ntc) * BN;
  // Nr % 256 == 128 (the 50304-row lm_head / embedding gradient): the last row tile has
  // 128 valid dW rows -- its other half re-reads valid columns (no out-of-bounds reads
  // at the end of dY) and stores nothing (wm >= 2 is wave-uniform)
  const bool half_tile = r0 + 256 > Nr;
  const int npair = T / (2 * GW_BK);
  const int p0 = (int)(((long)split * npair) / splits), p1 = (int)(((long)(split + 1) * npair) / splits);
  float* const dst = out + (accumulate ? 0 : (size_t)split * Nr * Nc) + (size_t)r0 * Nc + c0;
  gw_segment<HK, BN>(lds, dY, X, r0, c0, 2 * p0, 2 * (p1 - p0), half_tile, ldy, ldx, dst, Nc, accumulate != 0);
}

// ---------------------------------------------------------------- stream-K (round 3)
// The split-K grid above runs tiles x splits workgroups in whole rounds of 256, each
// round ending in a chip-wide burst of fp32 partial stores, and writes s full partial
// copies of dW for the fixed-order sum.  Stream-K instead gives each of G = Gc x ntc
// resident workgroups an equal contiguous share of the (row tile, 128-token pair)
// iteration space of ONE column tile c (column-major over c, so the ntc workgroups with
// the same share index g read the same dY rows at the same time -- they are dispatched
// together on one XCD, ids 8 * (ntc * (g / 8) + c) + g % 8, as above).  A share crossing
// row tiles runs one segment per row tile: a segment covering a whole tile accumulates
// straight into dW, a partial one writes its fp32 tile to its slot part[c][g][j] (j = row
// tile - the share's first row tile), and k_wgrad_sk_fix adds the slots of every split
// tile into dW in increasing g -- a fixed order, bitwise reproducible, no atomics.
struct GwSk {
  int npair, nrt, Wc, Gc, maxseg;
  __device__ __forceinline__ long s_of(int g) const { return (long)g * Wc / Gc; }  // first iteration of share g
  // share containing iteration i
  __device__ __forceinline__ int g_of(long i) const {
    int g = (int)((i * Gc) / Wc);
    while (g + 1 < Gc && s_of(g + 1) <= i) ++g;
    while (g > 0 && s_of(g) > i) --g;
    return g;
  }
};

template <int HK, int BN = 192>
__global__ __launch_bounds__(512, 1) void k_gemm_wgrad_sk(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                                          float* __restrict__ dW, float* __restrict__ part, int Nr,
                                                          int Nc, int ldy, int ldx, GwSk sk) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * GW_BUF];
  const int ntc = Nc / BN;
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int c = q % ntc, g = (q / ntc) * 8 + xcd;
  if (g >= sk.Gc) return;  // padding (uniform, before any barrier)
  const int c0 = c * BN;
  const long e = sk.s_of(g + 1);
  long i = sk.s_of(g);
  const int rt_first = (int)(i / sk.npair);
  while (i < e) {  // wave-uniform
    const int rt = (int)(i / sk.npair), p0 = (int)(i - (long)rt * sk.npair);
    const int p1 = (int)min((long)sk.npair, p0 + (e - i));
    const int r0 = rt * 256;
    const bool whole = p0 == 0 && p1 == sk.npair;
    float* dst = whole ? dW + (size_t)r0 * Nc + c0
                       : part + (((size_t)c * sk.Gc + g) * sk.maxseg + (rt - rt_first)) * (256 * BN);
    gw_segment<HK, BN>(lds, dY, X, r0, c0, 2 * p0, 2 * (p1 - p0), r0 + 256 > Nr, ldy, ldx, dst, whole ? Nc : BN, whole);
    i += p1 - p0;
  }
}

// dW tile (rt, c) += sum over the shares g_lo..g_hi that split it of their slots, in
// increasing g.  Grid: (GW_FIX_SPLIT, tiles); each block sums 1/GW_FIX_SPLIT of the tile.
// The slot index of every share is computed once per block (64-bit divisions) into LDS.
constexpr int GW_FIX_SPLIT = 48;
template <int BN = 192>
__global__ __launch_bounds__(256) void k_wgrad_sk_fix(const float* __restrict__ part, float* __restrict__ dW, int Nr,
                                                      int Nc, GwSk sk) {
  __shared__ int jt[256];
  const int ntc = Nc / BN;
  const int tile = blockIdx.y, rt = tile / ntc, c = tile - rt * ntc;
  const long i0 = (long)rt * sk.npair, i1 = i0 + sk.npair - 1;
  const int g_lo = sk.g_of(i0), g_hi = sk.g_of(i1);
  if (g_lo == g_hi) return;  // one share ran the whole tile into dW
  const int nsh = g_hi - g_lo + 1;
  for (int t = threadIdx.x; t < nsh && t < 256; t += 256) jt[t] = rt - (int)(sk.s_of(g_lo + t) / sk.npair);
  __syncthreads();
  const int rows = min(256, Nr - rt * 256);
  const float4* pc = reinterpret_cast<const float4*>(part) + ((size_t)c * sk.Gc + g_lo) * sk.maxseg * (256 * BN / 4);
  const size_t gstride = (size_t)sk.maxseg * (256 * BN / 4);  // float4s between consecutive shares' slot 0
  for (int k = blockIdx.x * 256 + threadIdx.x; k < 256 * BN / 4; k += gridDim.x * 256) {
    const int r = (k * 4) / BN, col = (k * 4) % BN;
    if (r >= rows) break;  // k grows with r: the rest of this thread's elements are past Nr too
    float4* d = reinterpret_cast<float4*>(dW + (size_t)(rt * 256 + r) * Nc + c * BN + col);
    float4 a = *d;
    for (int t = 0; t < nsh; ++t) {
      const int j = t < 256 ? jt[t] : rt - (int)(sk.s_of(g_lo + t) / sk.npair);
      const float4 p = pc[t * gstride + (size_t)j * (256 * BN / 4) + k];
      a.x += p.x;
      a.y += p.y;
      a.z += p.z;
      a.w += p.w;
    }
    *d = a;
  }
}

// dW column tile of a shape: 192 when it divides Nc, else 128 (0 = neither tiles)
static inline int gw_bn(int Nc) { return Nc % 192 == 0 ? 192 : (Nc % 128 == 0 ? 128 : 0); }

static inline GwSk gw_sk_plan(int T, int Nr, int Nc, int Gc_req) {
  GwSk sk{};
  sk.npair = T / 128;
  sk.nrt = (Nr + 255) / 256;
  sk.Wc = sk.nrt * sk.npair;
  const int ntc = Nc / gw_bn(Nc);
  int Gc = Gc_req > 0 ? Gc_req : 256 / ntc;
  Gc = Gc < 1 ? 1 : (Gc > sk.Wc ? sk.Wc : Gc);
  sk.Gc = Gc;
  // a share of ceil(Wc / Gc) iterations touches at most ceil(share / npair) + 1 row tiles
  const int share = (sk.Wc + Gc - 1) / Gc;
  sk.maxseg = (share + sk.npair - 1) / sk.npair + 1;
  return sk;
}

// Floats of scratch the stream-K weight gradient needs (0 = shape does not tile).
DLT_API long dlt_gemm_wgrad_sk_scratch(int T, int Nr, int Nc, int Gc) {
  if (T <= 0 || T % 128 || Nr % 128 || !gw_bn(Nc)) return 0;
  const int bn = gw_bn(Nc);
  const GwSk sk = gw_sk_plan(T, Nr, Nc, Gc);
  return (long)(Nc / bn) * sk.Gc * sk.maxseg * 256 * bn;
}

// dW[Nr, Nc] (fp32) += dY[T, Nr]^T . X[T, Nc], stream-K over Gc shares per column tile
// (Gc <= 0: 256 / column tiles, one workgroup per CU); `part` holds
// dlt_gemm_wgrad_sk_scratch() floats.  Deterministic (fixed-order fixup).  hk: operand
// format (0 bf16, 1 fp16).
DLT_API int dlt_gemm_wgrad_sk(const bf16_t* dY, const bf16_t* X, float* dW, float* part, int T, int Nr, int Nc,
                              int ldy, int ldx, int Gc, int hk, hipStream_t st) {
  const int bn = gw_bn(Nc);
  if (T <= 0 || T % 128 || Nr % 128 || !bn || (ldy | ldx) % 8 || !dW || !part) return -1;
  const GwSk sk = gw_sk_plan(T, Nr, Nc, Gc);
  const int ntc = Nc / bn;
  const int grid = ((sk.Gc + 7) / 8) * 8 * ntc;
  if (bn == 192) {
    DLT_HK_DISPATCH(hk, k_gemm_wgrad_sk<HKC, 192><<<grid, 512, 0, st>>>(dY, X, dW, part, Nr, Nc, ldy, ldx, sk));
  } else {
    DLT_HK_DISPATCH(hk, k_gemm_wgrad_sk<HKC, 128><<<grid, 512, 0, st>>>(dY, X, dW, part, Nr, Nc, ldy, ldx, sk));
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (bn == 192) k_wgrad_sk_fix<192><<<dim3(GW_FIX_SPLIT, sk.nrt * ntc), 256, 0, st>>>(part, dW, Nr, Nc, sk);
  else k_wgrad_sk_fix<128><<<dim3(GW_FIX_SPLIT, sk.nrt * ntc), 256, 0, st>>>(part, dW, Nr, Nc, sk);
  DLT_CHECK_LAUNCH();
}

// dW[Nr, Nc] (fp32) += dY[T, Nr]^T . X[T, Nc].  splits == 1: accumulated in place; splits
// > 1: the fp32 partials go to `part` [splits, Nr, Nc] (the caller sums them into dW in a
// fixed order).  Returns -1 (nothing launched) for shapes outside the tiling.  hk:
// operand format (0 bf16, 1 fp16).
DLT_API int dlt_gemm_wgrad(const bf16_t* dY, const bf16_t* X, float* dW, float* part, int T, int Nr, int Nc, int ldy,
                           int ldx, int splits, int hk, hipStream_t st) {
  const int bn = gw_bn(Nc);
  if (T <= 0 || T % 128 || Nr % 128 || !bn || (ldy | ldx) % 8 || splits < 1 || splits > T / 128) return -1;
  if (splits > 1 && part == nullptr) return -1;
  const int units = ((Nr + 255) / 256) * splits;  // (row tile, split) pairs, padded to 8s
  const int grid = ((units + 7) / 8) * 8 * (Nc / bn);
  if (bn == 192) {
    DLT_HK_DISPATCH(hk, k_gemm_wgrad<HKC, 192><<<grid, 512, 0, st>>>(dY, X, splits > 1 ? part : dW, T, Nr, Nc, ldy,
                                                                    ldx, splits, splits > 1 ? 0 : 1));
  } else {
    DLT_HK_DISPATCH(hk, k_gemm_wgrad<HKC, 128><<<grid, 512, 0, st>>>(dY, X, splits > 1 ? part : dW, T, Nr, Nc, ldy,
                                                                    ldx, splits, splits > 1 ? 0 : 1));
  }
  DLT_CHECK_LAUNCH();
}
