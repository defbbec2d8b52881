// Causal flash attention (head_dim 64 or 128: template parameter D) with in-kernel
// dropout for gfx950 MFMA.
//
// Replaces the reference's naive attention (gpt.py:230-234: Q@K^T, triu mask,
// fp32 softmax, bernoulli dropout, @V -- a [B,nh,S,S] score tensor per layer) and
// the SDPA path (gpt.py:199-206).  SURVEY §2.5 K5/K6.
//
// Design (CDNA4-first, see docs/KERNELS.md):
//  * v_mfma_f32_32x32x16_bf16 everywhere, accumulators in arch VGPRs
//    (-mllvm -amdgpu-mfma-vgpr-form: no v_accvgpr copies around the softmax).
//  * "Swapped" products put the softmax row on the lane: S^T = K.Q^T leaves one
//    query per lane with its keys in 16 accumulator registers, so row max / row sum
//    are in-lane plus one xor-32 swap, and the accumulator IS the B operand of the
//    next product (O^T = V^T.P^T) -- P never touches LDS.
//  * V / dO / Q / K^T operands are read with ds_read_b64_tr_b16 (hardware transpose).
//  * K/V (fwd, dQ) and Q/dO (dK/dV) tiles are register-staged into XOR-swizzled LDS,
//    double buffered: global loads of tile t+1 are issued before the MFMAs of tile t
//    and written to LDS after them (issue-early / write-late), one barrier per tile.
//  * Wave-uniform control: the wave index goes through readfirstlane, and each tile
//    is dispatched to a MASKED (diagonal / ragged) or UNMASKED instantiation, so the
//    hot loop has no exec-mask divergence and no per-element mask selects.
//  * Dropout: a VALU kernel hashes the keep decisions once (one lowbias32 per two
//    keys) into bitmasks in two layouts, row-major [bh][q][S/32] for the kernels
//    whose lanes are queries (fwd, dQ) and transposed [bh][k][S/32] for dK/dV whose
//    lanes are keys -- every MFMA kernel fetches ONE 32-bit word per lane per 32x32
//    sub-tile (2 x 12.6 MB per layer at B8 S1024 nh12).
//  * Backward = 2 kernels: dQ (recomputes S, dP; also emits Delta = rowsum(dO*O)),
//    then dK/dV (accumulated in registers) -- no fp32 atomics anywhere.  Causal
//    tile skipping; workgroups process paired items of equal total length.
//
// Layouts: q, k, v, dq, dk, dv: strided views -- head-major [B*nh, S, 64] or the
// packed [B*S, 3, nh, 64] QKV GEMM output (see dlt_attn_fwd_ex); o, do: [B, S, nh, 64]
// bf16 (= the [M, H] GEMM layout);  lse, delta: [B*nh, S] fp32 (natural-log lse).
#include "common.h"

#ifndef DLT_ATTN_KREAD_ASM
#define DLT_ATTN_KREAD_ASM 1
#endif

#include <type_traits>

#define KVB 64     // keys per staged tile (fwd / dQ)
#define RB 64      // rows (queries for fwd / dQ, keys for dK/dV) per work item: 2 waves x 32
#define QSTEP 64   // queries per staged tile (dK/dV)
#define NT 128     // threads per workgroup
#define LOG2E 1.44269504088896340736f

typedef __attribute__((address_space(3))) shortx4_t lds_shortx4_t;
typedef short shortx8_t __attribute__((ext_vector_type(8)));

// LDS tile: [64 rows][D bf16].  D = 64: 128-B rows, 16-B chunk c of row r stored at
// chunk c ^ ((r >> 1) & 7) -- row pairs fill the 64 banks, so 16 consecutive rows of a
// ds_read_b128 row-fragment read are conflict-free.  D = 128: 256-B rows (every row
// starts at bank 0), chunk c ^ (r & 15) gives 16 consecutive rows 16 distinct chunks.
template <int D>
__device__ __forceinline__ int swz_x(int row) { return D == 64 ? ((row >> 1) & 7) : (row & 15); }
template <int D>
__device__ __forceinline__ int swz_off(int row, int col) {
  return row * D + ((((col >> 3) ^ swz_x<D>(row))) << 3) + (col & 7);
}

template <int D>
__device__ __forceinline__ bf16x8_t lds_row8(const bf16_t* T, int row, int col) {
  return *reinterpret_cast<const bf16x8_t*>(T + swz_off<D>(row, col));
}

template <int D>
__device__ __forceinline__ shortx4_t lds_tr4(const bf16_t* T, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4_t*)(T + swz_off<D>(row, col)));
}

// A operand A[d][k] (k = rows of T) in the permuted k order that matches accumulator
// registers 8s..8s+7 used as the B operand: element j of lane-half h <-> row
// 16*kk + 8*(j>>2) + 4*h + (j&3)  (cdna_hip_programming.md §3).
template <int D>
__device__ __forceinline__ bf16x8_t tr_frag(const bf16_t* T, int kk, int dt, int lane) {
  const int h = lane >> 5, i = lane & 15;
  const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const int r1 = 16 * kk + 4 * h + (i >> 2);
  const shortx4_t a = lds_tr4<D>(T, r1, col);
  const shortx4_t b = lds_tr4<D>(T, r1 + 8, col);
  shortx8_t c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, c);
}

// The same fragment read through inline asm.  hipcc conservatively drains vmcnt(0)
// before any ds_read_b64_tr_b16 *intrinsic* while a global_load_lds is in flight
// (it cannot prove the DMA target and the read disjoint), which serialises the next
// tile's LDS-DMA with this tile's compute.  Asm reads are invisible to that alias
// check; the protocol that makes them safe is explicit: every tile step ends with
// `s_waitcnt vmcnt(0)` + barrier (tile_barrier), so a tile is complete before any
// wave reads it, and tr_wait() retires the reads before their registers are used.
template <int D>
__device__ __forceinline__ shortx4_t lds_tr4_asm(const bf16_t* T, int row, int col) {
  shortx4_t r;
  const uint32_t addr = (uint32_t)(uintptr_t)(T + swz_off<D>(row, col));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int D>
__device__ __forceinline__ bf16x8_t tr_frag_asm(const bf16_t* T, int kk, int dt, int lane) {
  const int h = lane >> 5, i = lane & 15;
  const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const int r1 = 16 * kk + 4 * h + (i >> 2);
  const shortx4_t a = lds_tr4_asm<D>(T, r1, col);
  const shortx4_t b = lds_tr4_asm<D>(T, r1 + 8, col);
  shortx8_t c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, c);
}
// Row-fragment read through inline asm (see lds_tr4_asm for the protocol), so several
// reads can be in flight under one counted wait (the intrinsic form drew one
// lgkmcnt(0) per MFMA pair).
template <int D>
__device__ __forceinline__ bf16x8_t lds_row8_asm(const bf16_t* T, int row, int col) {
  bf16x8_t r;
  const uint32_t addr = (uint32_t)(uintptr_t)(T + swz_off<D>(row, col));
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
// Oldest four of eight outstanding LDS reads retired (LDS returns in order; no SMEM
// load is issued inside a tile step).
__device__ __forceinline__ void lgkm_wait4(bf16x8_t& a, bf16x8_t& b, bf16x8_t& c, bf16x8_t& d) {
  asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}
// D = 128 forms: the oldest eight of sixteen reads retired; pin4 keeps four more
// fragments' consumers below the preceding wait (volatile asm stays in order).
__device__ __forceinline__ void lgkm_wait8(bf16x8_t& a, bf16x8_t& b, bf16x8_t& c, bf16x8_t& d) {
  asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}
__device__ __forceinline__ void pin4(bf16x8_t& a, bf16x8_t& b, bf16x8_t& c, bf16x8_t& d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
// Retire every outstanding LDS read, holding the consumers of all N fragments below it.
template <int N>
__device__ __forceinline__ void tr_wait_all(bf16x8_t (&f)[N]) {
  static_assert(N % 4 == 0, "groups of four");
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3])::"memory");
#pragma unroll
  for (int j = 4; j < N; j += 4) pin4(f[j], f[j + 1], f[j + 2], f[j + 3]);
}
__device__ __forceinline__ float max16(const floatx16_t& a) {
  const float m0 = fmaxf(fmaxf(a[0], a[1]), a[2]), m1 = fmaxf(fmaxf(a[3], a[4]), a[5]);
  const float m2 = fmaxf(fmaxf(a[6], a[7]), a[8]), m3 = fmaxf(fmaxf(a[9], a[10]), a[11]);
  const float m4 = fmaxf(fmaxf(a[12], a[13]), a[14]);
  return fmaxf(fmaxf(fmaxf(m0, m1), m2), fmaxf(fmaxf(m3, m4), a[15]));
}
// Retire outstanding LDS reads; the fragments are in/out operands so no consumer can
// be scheduled above the wait.
__device__ __forceinline__ void tr_wait(bf16x8_t& a, bf16x8_t& b, bf16x8_t& c, bf16x8_t& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}
// End of a tile step: this wave's LDS-DMA writes have landed, then the workgroup syncs.
__device__ __forceinline__ void tile_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Accumulator registers 8s..8s+7 as a bf16 MFMA operand: one v_cvt_pk_bf16_f32 per
// pair (an element-wise cast after a select made hipcc emit one cvt per element plus
// a v_perm per pair).
typedef float floatx8_t __attribute__((ext_vector_type(8)));
// HK = 1 (fp16 activations): the same registers as fp16 (RNE), kept in the bf16x8_t
// container type -- fragments are raw 16-byte operands; only mfma<HK> reads their format.
template <int HK = 0>
__device__ __forceinline__ bf16x8_t acc_frag(const floatx16_t& acc, int s) {
  const floatx8_t f = s ? acc.s89abcdef : acc.s01234567;
  if constexpr (HK == 0) return __builtin_convertvector(f, bf16x8_t);
  else return __builtin_bit_cast(bf16x8_t, __builtin_convertvector(f, f16x8_t));
}
// element j of a 16-bit fragment as float
template <int HK>
__device__ __forceinline__ float frag_f(const bf16x8_t& v, int j) {
  if constexpr (HK == 0) return (float)v[j];
  else return (float)__builtin_bit_cast(f16x8_t, v)[j];
}

// Dropout select on the fp32 bit pattern: all-ones / all-zeros from keep bit `bit` of
// `word` (v_bfe_i32), then one AND -- 2 VALU per element instead of and + cmp +
// cndmask.  A dropped element becomes +0.0f.
__device__ __forceinline__ uint32_t keep_ones(uint32_t word, int bit) {
  uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)word, bit, 1);
  // Empty asm (no instruction, so nothing for the hazard recognizer to miss): hides
  // that m is 0 / ~0, which stops LLVM from rewriting bfe + and as and + cmp + cndmask.
  asm("" : "+v"(m));
  return m;
}
__device__ __forceinline__ float keep_and(float x, uint32_t ones) {
#ifdef DLT_ATTN_NOSEL  // diagnostic upper bound only (tools/ab): drops nothing, wrong numerics
  return x;
#endif
  return __uint_as_float(__float_as_uint(x) & ones);
}

template <int HK = 0>
__device__ __forceinline__ floatx16_t mfma(const bf16x8_t& a, const bf16x8_t& b, const floatx16_t& c) {
  if constexpr (HK == 0) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// row (within a 32x32 tile) of accumulator register i for lane-half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ floatx16_t zero16() {
  floatx16_t z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// Direct global->LDS tile copy (global_load_lds_dwordx4, no staging registers): one
// wave-instruction writes 1 KiB = 1024 / (2D) rows contiguously (lane l -> row
// l / (D/8), 16-B slot l % (D/8)), so the XOR swizzle is applied on the SOURCE
// address: slot s of row r holds global chunk s ^ swz_x(r), exactly the image
// swz_off() reads.  64 rows = 8 (D = 64) or 16 (D = 128) instructions, split over the
// 2 waves.  Completion is tracked by vmcnt; the __syncthreads() that ends every tile
// step waits for it.
typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef const __attribute__((address_space(1))) void* gbl_cvptr_t;
template <int D>
__device__ __forceinline__ void glds_tile(const bf16_t* __restrict__ base, int row0, int S, int rstride, bf16_t* T,
                                          int wid, int lane) {
  // 32-bit offsets (a head's rows span < 4 GB) on the wave-uniform base: the DMA takes
  // the saddr form and no 64-bit address arithmetic runs per tile (fwd / dQ).
  constexpr int CPR = D / 8, RPI = 64 / CPR, NI = 32 / RPI;  // chunks / row, rows / instr, instr / wave
  const char* b = reinterpret_cast<const char*>(base);
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int rr = (wid * NI + j) * RPI;  // first row of this 1 KiB piece (wave-uniform)
    const int row = rr + lane / CPR;
    const int c = (lane % CPR) ^ swz_x<D>(row);
    const uint32_t off = (uint32_t)(min(row0 + row, S - 1) * rstride + c * 8) * 2u;
    __builtin_amdgcn_global_load_lds((gbl_cvptr_t)(b + off), (lds_vptr_t)(T + rr * D), 16, 0, 0);
  }
}
// The same copy with 64-bit row addressing: fewer live registers in dK/dV, which stages
// two operands with different row strides and sits at the VGPR limit.
template <int D>
__device__ __forceinline__ void glds_tile64(const bf16_t* __restrict__ base, int row0, int S, int rstride, bf16_t* T,
                                            int wid, int lane) {
  constexpr int CPR = D / 8, RPI = 64 / CPR, NI = 32 / RPI;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int rr = (wid * NI + j) * RPI;
    const int row = rr + lane / CPR;
    const int c = (lane % CPR) ^ swz_x<D>(row);
    const bf16_t* g = base + (size_t)min(row0 + row, S - 1) * rstride + c * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvptr_t)g, (lds_vptr_t)(T + rr * D), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8_t load_row8(const bf16_t* __restrict__ p, bool ok) {
  bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(p);
  if (!ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
  }
  return v;
}

// ============================================================================ dropout bits
// Keep-bit words in two layouts (one hash per element pair, computed once):
//   mask [bh][w][q]  bit j = keep(q, key = 32w + j)   -- lane = query (fwd, dQ)
//   maskT[bh][w][k]  bit j = keep(q = 32w + j, key k) -- lane = key   (dK/dV)
// Word-major: the 32 lanes that write (here) or read (MFMA kernels: lane = row) one
// word index touch 128 contiguous bytes; the row-major [bh][q][w] layout made every
// lane's 4-byte access its own cache line (the store side cost ~3x the hashing).
// Only causal 32x32 tiles (key word <= query band) exist.  One half-wave per tile:
// lane l hashes row q = 32r + l (16 hashes -> its row word), then a 5-stage butterfly
// bit transpose gives lane j the column word of key 32w + j.
// Pure VALU, so the MFMA kernels only test bits instead of hashing at 2 waves/SIMD.
// Instruction budget (S % 32 == 0, the fast path): 11 VALU per hash -- the pair index
// is one xor (the row word's 16 pair indices differ from its first only in their low
// 4 bits), and each keep bit is the carry of (16 random bits in the high half) +
// (65536 - thr) << 16, shifted into the word by v_addc (no compare / select / or per
// bit); the transpose is branch-free (ds_swizzle + alignbit + bfi per stage).  Round 4
// form: ~32 VALU per hash (compare + s_nop + select per bit, divergent transpose).

// word = 2 * word + carry(v + c16): shifts in keep = (high 16 bits of v) >= thr at bit 0
// (c16 = (65536 - thr) << 16; the low half of c16 is zero, so v's low half never carries)
__device__ __forceinline__ uint32_t keep_shift_in(uint32_t word, uint32_t v, uint32_t c16) {
  uint32_t sum;  // discarded: only the carry is used
  asm("v_add_co_u32 %1, vcc, %2, %3\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
      : "+v"(word), "=&v"(sum)
      : "s"(c16), "v"(v)
      : "vcc");
  return word;
}
// (x ^ (x >> 16)) << 16: the low 16 bits of lowbias32's last step, in the high half
__device__ __forceinline__ uint32_t lo16_hi(uint32_t x) {
  uint32_t z;
  asm("v_xor_b32_sdwa %0, %1, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1"
      : "=v"(z)
      : "v"(x));
  return z;
}
// lane l ^ d within 32-lane groups (ds_swizzle bitmask mode: and 0x1f, xor d)
template <int d>
__device__ __forceinline__ uint32_t swz_xor(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1f | (d << 10));
}
template <int d>
__device__ __forceinline__ uint32_t bt_stage(uint32_t col, int l) {
  // lanes with bit d clear keep the m-bits of their word and take the partner's m-bits
  // shifted up by d (rotl d, the wrapped bits land in m and are dropped); lanes with
  // bit d set keep ~m and take the partner's ~m-bits shifted down (rotr d)
  constexpr uint32_t m = d == 16 ? 0x0000FFFFu : d == 8 ? 0x00FF00FFu : d == 4 ? 0x0F0F0F0Fu : d == 2 ? 0x33333333u
                                                                                               : 0x55555555u;
  const uint32_t y = swz_xor<d>(col);
  const bool up = (l & d) == 0;
  const uint32_t r = __builtin_amdgcn_alignbit(y, y, up ? 32 - d : d);
  const uint32_t keep = up ? m : ~m;
  return (col & keep) | (r & ~keep);
}

__global__ __launch_bounds__(256) void k_dropout_bits(uint32_t* __restrict__ mask, uint32_t* __restrict__ maskT,
                                                      int BH, int S, uint32_t key, uint32_t thr) {
  const int W = (S + 31) >> 5;  // words per row == number of 32-row bands
  const int bh = blockIdx.y;
  const int lane = threadIdx.x & 63, l = lane & 31;
  const int tile = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);  // one tile per half-wave
  const int ntiles = W * (W + 1) / 2;
  const bool active = tile < ntiles;
  // tile -> (band r, word w <= r): band r starts at tile r(r+1)/2; the float root is
  // within one of r for any realistic S, corrected once each way without loops
  int r = (int)((sqrtf(8.f * (float)tile + 1.f) - 1.f) * 0.5f);
  r += ((r + 1) * (r + 2) / 2 <= tile) ? 1 : 0;
  r -= (r * (r + 1) / 2 > tile) ? 1 : 0;
  const int w = tile - r * (r + 1) / 2;
  const int q = r * 32 + l;
  const uint32_t kbh = lowbias32(key + (uint32_t)bh * 0x9E3779B9u);
  uint32_t word = 0;
  if (active && q < S) {
    const uint32_t base = (uint32_t)q * (uint32_t)S + (uint32_t)(w * 32);
    if ((S & 31) == 0) {
      // base % 32 == 0: pair index base/2 + m has m in the 4 low bits, which base/2 lacks
      const uint32_t kx = kbh ^ (base >> 1);
      const uint32_t c16 = (65536u - thr) << 16;
#pragma unroll
      for (int m = 15; m >= 0; --m) {  // bits shift in from the top element down
        uint32_t x = kx ^ (uint32_t)m;
        x ^= x >> 16;
        x *= 0x7feb352du;
        x ^= x >> 15;
        x *= 0x846ca68bu;
        word = keep_shift_in(word, x, c16);            // element 2m + 1: high 16 bits
        word = keep_shift_in(word, lo16_hi(x), c16);  // element 2m: low 16 bits
      }
    } else {
      const int nk = min(32, S - w * 32);
      for (int j = 0; j < nk; ++j) {
        const uint32_t flat = base + (uint32_t)j;
        const uint32_t hsh = lowbias32(kbh ^ (flat >> 1));
        const uint32_t bits = (flat & 1u) ? (hsh >> 16) : (hsh & 0xffffu);
        word |= (uint32_t)(bits >= thr) << j;
      }
    }
    mask[((size_t)bh * W + w) * S + q] = word;  // word-major: the half-wave's 32 rows are contiguous
  }
  // 32x32 bit transpose within each half-wave (lane l holds row l; afterwards lane j
  // holds column j).  Every lane runs it (inactive lanes carry zeros) so the swizzles see
  // a full group.
  uint32_t col = word;
  col = bt_stage<16>(col, l);
  col = bt_stage<8>(col, l);
  col = bt_stage<4>(col, l);
  col = bt_stage<2>(col, l);
  col = bt_stage<1>(col, l);
  const int kk = w * 32 + l;
  if (active && kk < S) maskT[((size_t)bh * W + r) * S + kk] = col;
}

// ============================================================================ work map
// The MFMA kernels run a 1-D grid of (head, item-pair) work items.  The dispatcher deals
// consecutive workgroup ids round-robin to the 8 XCDs, each with its own 4 MB L2; with
// the natural order (pair fastest) XCD x would get pair x of EVERY head, so no two
// workgroups on an XCD share a K/V (fwd, dQ) or Q/dO (dK/dV) stream and every tile is
// fetched once per pair from the fabric.  The XCD-aware map gives each XCD a contiguous
// range of items instead -- all pairs of a head on one XCD, reading the head's tiles
// through the same L2 (bijective for any grid size, like the GEMM's tile map).
__device__ __forceinline__ bool work_item(int nrb, int sched, int& bh, int& pair) {
  const int bid = blockIdx.x;
  if (sched & 2) {
    // LPT: one 64-row item per workgroup, longest first (block ids ascend in dispatch
    // order), so short items fill the slots the long ones leave -- many more, shorter
    // waves than the pairing.  bid % 8 == bh % 8 when B*nh % 8 == 0: a head stays on
    // one XCD (its K/V or Q/dO tiles through one L2).
    const int BH = gridDim.x / nrb;
    pair = bid / BH;  // rank: 0 = longest item
    bh = bid - pair * BH;
    return true;
  }
  const int npairs = (nrb + 1) / 2;
  int wg = bid;
  if (sched & 1) {
    const int nwg = gridDim.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  }
  bh = wg / npairs;
  pair = wg - bh * npairs;
  return false;
}

// ============================================================================ forward
// Cross-half (lane i <-> i^32) exchange without LDS: v_permlane32_swap (CDNA4).
__device__ __forceinline__ float xhalf_max(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// 16-byte row stores from the split-lane accumulator layout.  Lane (row, h) holds dims
// 32dt + 8g + 4h + [0, 4) (w[dt][g], 4 bf16 = 2 dwords).  One v_permlane32_swap of the
// (g = 2m, 2m + 1) pair -- own g = 2m stays in the low lanes' vdst, the high lanes' g = 2m
// lands there; own g = 2m + 1 stays in the high lanes' vsrc -- leaves lane h holding
// dims 16m + 8h + [0, 8): 4 dwordx4 stores per row instead of 8 dwordx2 (the epilogue's
// store issue is the tail of every work item).
template <int D>
__device__ __forceinline__ void store_row16(bf16_t* __restrict__ row, const uint2 (&w)[D / 32][4], int h) {
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const auto rx = __builtin_amdgcn_permlane32_swap(w[dt][2 * m].x, w[dt][2 * m + 1].x, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(w[dt][2 * m].y, w[dt][2 * m + 1].y, false, false);
      *reinterpret_cast<uint4*>(row + 32 * dt + 16 * m + 8 * h) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
}

// Rescale threshold (log2 units): the running max is only moved when some row's max
// grew by more than 2^RESCALE_LOG2 (P is then bounded by 2^8 = 256 instead of 1,
// exact in fp32 l/O and the same relative bf16 precision for P).  Almost every
// rescale after a row's first tile is skipped.
#define RESCALE_LOG2 8.0f

template <int D>
struct FwdState {
  floatx16_t o[D / 32];
  float m, l;  // running max (raw score units) and per-lane partial row sum
};

template <bool MASK, bool DROP, int HK, int D>
__device__ __forceinline__ void fwd_tile(FwdState<D>& fs, const bf16_t* Kt, const bf16_t* Vt,
                                         const bf16x8_t (&qf)[D / 16], int k0, int qa, int S, int lane, float c_log2,
                                         uint2 mw) {
  // One 64-key tile as ONE online-softmax step: S = K.Q^T of both 32-key halves first
  // (two independent MFMA chains), one row max / rescale decision for the tile, then
  // per half exp -> dropout -> P.V; the second half's softmax VALU runs while the
  // first half's P.V MFMAs execute.  The row sum uses two partial sums (the single
  // running sum was a 16-deep dependent add chain per half).
  const int h = lane >> 5, ql = lane & 31;
  // keep-bit words of this tile (prefetched with the previous tile's staging loads,
  // so no vmcnt wait lands inside the tile); this lane-half's 16 bits per half-tile
  // sit at (i&3) + 8(i>>2)
  const uint32_t words[2] = {mw.x >> (4 * h), mw.y >> (4 * h)};
  constexpr int NS = D / 16;  // 16-dim contraction steps of S = K.Q^T
  floatx16_t sacc[2];
  {
    bf16x8_t kf[2][NS];
#if DLT_ATTN_KREAD_ASM
    // all K fragments of the tile in flight at once, one counted wait per half
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < NS; ++s) kf[t][s] = lds_row8_asm<D>(Kt, 32 * t + ql, 16 * s + 8 * h);
    if constexpr (D == 64) {
      lgkm_wait4(kf[0][0], kf[0][1], kf[0][2], kf[0][3]);
    } else {
      lgkm_wait8(kf[0][0], kf[0][1], kf[0][2], kf[0][3]);
      pin4(kf[0][4], kf[0][5], kf[0][6], kf[0][7]);
    }
    sacc[0] = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) sacc[0] = mfma<HK>(kf[0][s], qf[s], sacc[0]);
    tr_wait_all(kf[1]);
    sacc[1] = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) sacc[1] = mfma<HK>(kf[1][s], qf[s], sacc[1]);
#else
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      kf[0][s] = lds_row8<D>(Kt, ql, 16 * s + 8 * h);
      kf[1][s] = lds_row8<D>(Kt, 32 + ql, 16 * s + 8 * h);
    }
    sacc[0] = zero16();
    sacc[1] = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      sacc[0] = mfma<HK>(kf[0][s], qf[s], sacc[0]);
      sacc[1] = mfma<HK>(kf[1][s], qf[s], sacc[1]);
    }
#endif
  }
  if (MASK) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ka = k0 + 32 * t + acc_row(i, h);
        sacc[t][i] = (ka > qa || ka >= S) ? -INFINITY : sacc[t][i];
      }
  }
  // row max as a depth-3 max3 tree per half (a linear fmaxf chain is 9 dependent ops)
  const float mx = xhalf_max(fmaxf(max16(sacc[0]), max16(sacc[1])));
  if (!__all((mx - fs.m) * c_log2 <= RESCALE_LOG2)) {  // rare: a row's max grew by > 2^8
    const float m_new = fmaxf(fs.m, mx);
    const float alpha = fast_exp2((fs.m - m_new) * c_log2);
    fs.m = m_new;
    fs.l *= alpha;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) fs.o[dt][i] *= alpha;
  }
  const float nmc = -fs.m * c_log2;
  float l0 = 0.f, l1 = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    bf16x8_t vf[2][D / 32];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) vf[kk][dt] = tr_frag_asm<D>(Vt, 2 * t + kk, dt, lane);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = fast_exp2(fmaf(sacc[t][i], c_log2, nmc));
      if (i & 1) l1 += p;
      else l0 += p;
      if (DROP) sacc[t][i] = keep_and(p, keep_ones(words[t], (i & 3) + 8 * (i >> 2)));  // 1/(1-p) at the end
      else sacc[t][i] = p;
    }
    if constexpr (D == 64) {
      tr_wait(vf[0][0], vf[0][1], vf[1][0], vf[1][1]);
    } else {
      tr_wait(vf[0][0], vf[0][1], vf[0][2], vf[0][3]);
      pin4(vf[1][0], vf[1][1], vf[1][2], vf[1][3]);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8_t pb = acc_frag<HK>(sacc[t], kk);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) fs.o[dt] = mfma<HK>(vf[kk][dt], pb, fs.o[dt]);
    }
  }
  fs.l += l0 + l1;
}

// Work decomposition (causal balance): a workgroup = 2 waves = one 64-query item.
// Default schedule (work_item, LPT): one item per workgroup, longest first, so the
// short items fill in behind the long ones.  Alternative (DLT_ATTN_SCHED=pair): each
// workgroup processes the PAIR of items (nrb-1-p, p), equal work per workgroup but
// only ~1.5 long waves per SIMD -- a half-empty last round at 2 waves/SIMD (PMC:
// ~1.1 resident waves per SIMD on average at B16).  Round 1 measured one item per
// workgroup in the NATURAL order 1.8x slower than the pairing (equal-length items
// stacked on a CU); longest-first does not stack them.
// Forward diagnostics (tools/cpp/attn_fwd_timing.cpp, -DDLT_ATTN_FWD_TIMING only): per
// wave, the shader cycles inside the tile compute and inside the per-tile DMA wait +
// barrier, and the tile count, written by lane 0 with vector stores.
#ifdef DLT_ATTN_FWD_TIMING
__device__ unsigned long long* g_attn_ftim;
#define FWD_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define FWD_ACC(c, w) (f_comp += (c), f_wait += (w), ++f_tiles)
#else
#define FWD_T(v) ((void)0)
#define FWD_ACC(c, w) ((void)0)
#endif

// D = 128 doubles the O accumulators and Q / K / V fragments: 256 VGPRs would spill,
// so its instantiation may take the whole 512-register file (one wave per SIMD).
#define ATTN_WAVES(D) __attribute__((amdgpu_waves_per_eu(D == 64 ? 2 : 1, 2)))
template <bool DROP, int HK, int D>
__global__ __launch_bounds__(NT) ATTN_WAVES(D) void k_attn_fwd(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                    const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                    float* __restrict__ lse, const uint32_t* __restrict__ mask,
                                                    int S, int nh, float c_log2, float dscale, long in_bs,
                                                    int in_hs, int in_rs, int xcd_map) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * KVB * D];  // [buf][K|V][64][D]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, ql = lane & 31;
  const int nrb = (S + RB - 1) / RB;
  int bh, pair;
  const bool lpt = work_item(nrb, xcd_map, bh, pair);
  const int b = bh / nh, head = bh % nh;
  const size_t hin = (size_t)b * in_bs + (size_t)head * in_hs;  // (b, head) base of q / k / v
  const int W = (S + 31) >> 5;
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using UNM = std::integral_constant<bool, false>;
  using MSK = std::integral_constant<bool, true>;
#ifdef DLT_ATTN_FWD_TIMING
  unsigned long long f_comp = 0, f_wait = 0, f_tiles = 0;
  const unsigned long long f_t0 = __builtin_amdgcn_s_memtime();
#endif

#pragma unroll 1
  for (int it = 0; it < 2; ++it) {
    const int qb = (lpt || it == 0) ? nrb - 1 - pair : pair;  // long item first
    if (it == 1 && (lpt || qb >= nrb - 1 - pair)) break;       // odd nrb: middle item once
    const int q0 = qb * RB + wid * 32;  // this wave's first query (wave-uniform)
    const int qa = q0 + ql;
    const uint32_t* mrow = mask ? mask + (size_t)bh * W * S + min(qa, S - 1) : nullptr;  // word j at mrow[j*S]

    bf16x8_t qf[D / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
      qf[s] = load_row8(q + hin + (size_t)min(qa, S - 1) * in_rs + 16 * s + 8 * h, qa < S);

    FwdState<D> fs;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) fs.o[dt] = zero16();
    fs.m = -INFINITY;
    fs.l = 0.f;

    const int nkv = (min(S, qb * RB + RB) + KVB - 1) / KVB;  // = qb + 1 except at a ragged end
    glds_tile<D>(k + hin, 0, S, in_rs, lds, wid, lane);
    glds_tile<D>(v + hin, 0, S, in_rs, lds + KVB * D, wid, lane);
    __syncthreads();

    // One K/V tile per step.  BUF is a compile-time LDS buffer index and MASKED a
    // compile-time tile kind: tiles kb < qb lie entirely below every query of the
    // item (straight-line unmasked loop, unrolled by two so every LDS address is
    // lane-base + immediate); tile qb holds the diagonal.
    uint2 mw_cur = make_uint2(0u, 0u), mw_next = make_uint2(0u, 0u);
    if (DROP) mw_cur = make_uint2(mrow[0], W > 1 ? mrow[S] : 0u);  // words of tile 0
    auto step = [&](auto bufc, auto maskc, int kb) {
      constexpr int BUF = decltype(bufc)::value;
      constexpr bool MASKED = decltype(maskc)::value;
      FWD_T(ta);
      const bool more = kb + 1 < nkv;
      if (more) {  // next tile straight into the other buffer (read by nobody since the last barrier)
        bf16_t* Kn = lds + (BUF ^ 1) * 2 * KVB * D;
        glds_tile<D>(k + hin, (kb + 1) * KVB, S, in_rs, Kn, wid, lane);
        glds_tile<D>(v + hin, (kb + 1) * KVB, S, in_rs, Kn + KVB * D, wid, lane);
        if (DROP) mw_next = make_uint2(mrow[(size_t)(2 * (kb + 1)) * S], 2 * (kb + 1) + 1 < W ? mrow[(size_t)(2 * (kb + 1) + 1) * S] : 0u);
      }
      const bf16_t* Kt = lds + BUF * 2 * KVB * D;
      const bf16_t* Vt = Kt + KVB * D;
      const int k0 = kb * KVB;
      if (!MASKED)
        fwd_tile<false, DROP, HK, D>(fs, Kt, Vt, qf, k0, qa, S, lane, c_log2, mw_cur);
      else if (k0 <= q0 + 31)
        fwd_tile<true, DROP, HK, D>(fs, Kt, Vt, qf, k0, qa, S, lane, c_log2, mw_cur);
      mw_cur = mw_next;
      FWD_T(tb);
      tile_barrier();
      FWD_T(tc);
      FWD_ACC(tb - ta, tc - tb);
    };
    const int nfull = min(qb, nkv);
    int kb = 0;
    for (; kb + 1 < nfull; kb += 2) {
      step(B0{}, UNM{}, kb);
      step(B1{}, UNM{}, kb + 1);
    }
    if (kb < nfull) {  // odd count: last unmasked tile in buffer 0, diagonal in buffer 1
      step(B0{}, UNM{}, kb);
      if (kb + 1 < nkv) step(B1{}, MSK{}, kb + 1);
    } else if (kb < nkv) {
      step(B0{}, MSK{}, kb);
    }

    const float l_tot = xhalf_sum(fs.l);
    const float inv_l = (DROP ? dscale : 1.f) / l_tot;
    if (qa < S) {
      if (h == 0) lse[(size_t)bh * S + qa] = fs.m * (c_log2 / LOG2E) + __logf(l_tot);
      bf16_t* orow = o + (((size_t)b * S + qa) * nh + head) * D;
      uint2 w[D / 32][4];
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u16x4 t;
#pragma unroll
          for (int e = 0; e < 4; ++e) t.v[e] = f2h<HK>(fs.o[dt][4 * g + e] * inv_l);
          w[dt][g] = __builtin_bit_cast(uint2, t);
        }
      store_row16<D>(orow, w, h);
    }
  }
#ifdef DLT_ATTN_FWD_TIMING
  const unsigned long long f_t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    unsigned long long* r = g_attn_ftim + ((size_t)blockIdx.x * 2 + wid) * 6;
    r[0] = f_t0; r[1] = f_t1; r[2] = f_comp; r[3] = f_wait; r[4] = f_tiles;
  }
#endif
}

// ============================================================================ backward
// Store one head row held in accumulators (element 4g+e of acc[dt] is dim
// 32*dt + 8*g + 4*h + e) times `sc`.  With RoPE tables the inverse NeoX rotation of
// position `pos` is applied first: the partner of dim j < 32 is j + 32, i.e. the same
// register of the other dt -- the rotation needs no data exchange.  (Replaces the
// separate repack kernel that read dq/dk back and wrote the packed [M, 3H] gradient.)
template <int HK, int D>
__device__ __forceinline__ void store_head_row(bf16_t* __restrict__ dst, const floatx16_t (&a)[D / 32], float sc, int h,
                                               const float* __restrict__ cosT, const float* __restrict__ sinT,
                                               int pos) {
  // dims of a[dt] element 4g + e: 32 dt + 8 g + 4 h + e; the RoPE partner of dim j < D/2
  // is j + D/2, register 4g + e of a[dt + D/64]
  constexpr int HP = D / 64;
  uint2 w[D / 32][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int dt = 0; dt < HP; ++dt) {
      u16x4 w0, w1;
      if (cosT) {
        const int ti = pos * (D / 2) + 32 * dt + 8 * g + 4 * h;
        const float4 c4 = *reinterpret_cast<const float4*>(cosT + ti);
        const float4 s4 = *reinterpret_cast<const float4*>(sinT + ti);
        const float cc[4] = {c4.x, c4.y, c4.z, c4.w}, ss[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x1 = a[dt][4 * g + e] * sc, x2 = a[dt + HP][4 * g + e] * sc;
          w0.v[e] = f2h<HK>(fmaf(x1, cc[e], x2 * ss[e]));
          w1.v[e] = f2h<HK>(fmaf(x2, cc[e], -x1 * ss[e]));
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w0.v[e] = f2h<HK>(a[dt][4 * g + e] * sc);
          w1.v[e] = f2h<HK>(a[dt + HP][4 * g + e] * sc);
        }
      }
      w[dt][g] = __builtin_bit_cast(uint2, w0);
      w[dt + HP][g] = __builtin_bit_cast(uint2, w1);
    }
  store_row16<D>(dst, w, h);
}

// Per-wave timestamps for tools/cpp/attn_timing.cpp (only with -DDLT_ATTN_TIMING):
// [workgroup][wave][8] shader-clock stamps written by lane 0 with vector stores.
#ifdef DLT_ATTN_TIMING
__device__ unsigned long long* g_attn_tim;
#define ATTN_STAMP(slot)                                                                           \
  do {                                                                                             \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                                   \
    if (lane == 0) g_attn_tim[((size_t)blockIdx.x * 2 + wid) * 8 + (slot)] = _t;                   \
  } while (0)
#else
#define ATTN_STAMP(slot) ((void)0)
#endif

// ---------------------------------------------------------------- dK / dV
// One workgroup per 128 keys (32 per wave); sweep query tiles of 64 (two 32-row
// sub-tiles).  Accumulators: S and dP with queries in registers, keys on lanes.
template <bool MASK, bool DROP, int HK, int D>
__device__ __forceinline__ void dkdv_subtile(floatx16_t (&dka)[D / 32], floatx16_t (&dva)[D / 32], const bf16_t* Qt,
                                             const bf16_t* Dt, const float* rl, const float* rd,
                                             uint32_t mw, const bf16x8_t (&kf)[D / 16], const bf16x8_t (&vf)[D / 16],
                                             int qs, int ka, int S, int lane, float c_log2, float dscale) {
  const int h = lane >> 5, kl = lane & 31;
  floatx16_t sacc = zero16(), pacc = zero16();
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    sacc = mfma<HK>(lds_row8<D>(Qt, kl, 16 * s + 8 * h), kf[s], sacc);
    pacc = mfma<HK>(lds_row8<D>(Dt, kl, 16 * s + 8 * h), vf[s], pacc);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 l4 = *reinterpret_cast<const float4*>(rl + 8 * g + 4 * h);
    const float4 d4 = *reinterpret_cast<const float4*>(rd + 8 * g + 4 * h);
    const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
    const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e;
      const int r = 8 * g + 4 * h + e;  // query row within the sub-tile
      float p = fast_exp2(fmaf(sacc[i], c_log2, -lv[e]));
      if (MASK) {
        const int qa = qs + r;
        p = (ka > qa || qa >= S || ka >= S) ? 0.f : p;
      }
      const float dp = pacc[i];
      if (DROP) {
        // dS = P o (s M o dP - Delta) = s (Pd o dP - P Delta / s) with Pd = M o P: the
        // dropped P that dV needs anyway, so the mask is applied once (4 VALU per
        // element instead of 5); rd holds Delta / s and s = 1/(1-p) is folded into the
        // dK and dV epilogues
        const uint32_t ones = keep_ones(mw, 8 * g + e);  // maskT word >> 4h: query qs + r
        const float pd = keep_and(p, ones);
        sacc[i] = pd;                          // dropped P -> dV
        pacc[i] = fmaf(pd, dp, -(p * dv[e]));  // dS / s   -> dK
      } else {
        sacc[i] = p;
        pacc[i] = p * (dp - dv[e]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8_t pb = acc_frag<HK>(sacc, s);
    const bf16x8_t sb = acc_frag<HK>(pacc, s);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      dva[dt] = mfma<HK>(tr_frag<D>(Dt, s, dt, lane), pb, dva[dt]);
      dka[dt] = mfma<HK>(tr_frag<D>(Qt, s, dt, lane), sb, dka[dt]);
    }
  }
}

// Work items: 64 keys (2 waves x 32); a workgroup processes the pair of key blocks
// (p, nrb-1-p) -- equal work per workgroup (see the forward).
template <bool DROP, int HK, int D>
__global__ __launch_bounds__(NT) ATTN_WAVES(D) void k_attn_bwd_dkdv(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                         const bf16_t* __restrict__ v,
                                                         const bf16_t* __restrict__ dout,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta,
                                                         const uint32_t* __restrict__ maskT, bf16_t* __restrict__ dk,
                                                         bf16_t* __restrict__ dv, int S, int nh, float c_log2,
                                                         float scale, float dscale, long in_bs, int in_hs, int in_rs,
                                                         long out_bs, int out_hs, int out_rs,
                                                         const float* __restrict__ cosT,
                                                         const float* __restrict__ sinT, int xcd_map) {
  // one LDS object (avoids hipcc's extra vmcnt waits with several __shared__ arrays)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * QSTEP * D * 2 + 2 * 2 * QSTEP * 4];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);                              // [buf][Q|dO][64][D]
  float* rowc = reinterpret_cast<float*>(smem + 2 * 2 * QSTEP * D * 2);       // [buf][lse2|delta][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, kl = lane & 31;
  ATTN_STAMP(0);
  const int nrb = (S + RB - 1) / RB;
  int bh, pair;
  const bool lpt = work_item(nrb, xcd_map, bh, pair);
  const int b = bh / nh, head = bh % nh;
  const size_t hin = (size_t)b * in_bs + (size_t)head * in_hs;     // q / k / v
  const size_t hout = (size_t)b * out_bs + (size_t)head * out_hs;  // dk / dv
  const int rstride = nh * D;
  const int W = (S + 31) >> 5;
  const int nqt = (S + QSTEP - 1) / QSTEP;
  const bf16_t* dob = dout + ((size_t)b * S * nh + head) * D;
  const float inv_dscale = 1.f / dscale;
  using UNM = std::integral_constant<bool, false>;
  using MSK = std::integral_constant<bool, true>;

#pragma unroll 1
  for (int it = 0; it < 2; ++it) {
    const int kblk = (lpt || it == 0) ? pair : nrb - 1 - pair;  // long item (early keys) first
    if (it == 1 && (lpt || kblk <= pair)) break;                 // odd nrb: middle item once
    const int k0 = kblk * RB + wid * 32;  // wave-uniform
    const int ka = k0 + kl;
    // this lane's key column of the transposed keep-bit mask: one word per 32 queries
    const uint32_t* mcol = DROP ? maskT + (size_t)bh * W * S + min(ka, S - 1) : nullptr;  // word j at mcol[j*S]

    bf16x8_t kf[D / 16], vf[D / 16];
    const int kc = min(ka, S - 1);
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      kf[s] = load_row8(k + hin + (size_t)kc * in_rs + 16 * s + 8 * h, ka < S);
      vf[s] = load_row8(v + hin + (size_t)kc * in_rs + 16 * s + 8 * h, ka < S);
    }
    floatx16_t dka[D / 32], dva[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) dka[dt] = dva[dt] = zero16();

    const int qt_begin = kblk;  // the 64-query tile holding this item's diagonal
    float rl = 0.f, rd = 0.f;
    uint2 mw_cur = make_uint2(0u, 0u), mw_next = make_uint2(0u, 0u);
    auto load_rows = [&](int t, int buf) {  // Q / dO tiles by LDS-DMA, row stats via registers
      glds_tile64<D>(q + hin, t * QSTEP, S, in_rs, lds + buf * 2 * QSTEP * D, wid, lane);
      glds_tile64<D>(dob, t * QSTEP, S, rstride, lds + buf * 2 * QSTEP * D + QSTEP * D, wid, lane);
      if (DROP) {  // this lane's two 32-query keep words of tile t (consumed one tile later)
        const int w0 = (t * QSTEP) >> 5;
        mw_next = make_uint2(mcol[(size_t)w0 * S], (w0 + 1 < W) ? mcol[(size_t)(w0 + 1) * S] : 0u);
      }
      if (tid < QSTEP) {
        const int qq = min(t * QSTEP + tid, S - 1);
        const bool ok = t * QSTEP + tid < S;
        rl = ok ? lse[(size_t)bh * S + qq] * LOG2E : 0.f;
        rd = ok ? delta[(size_t)bh * S + qq] * (DROP ? inv_dscale : 1.f) : 0.f;  // Delta / s (dkdv_subtile)
      }
    };
    auto store_rows = [&](int buf) {
      if (tid < QSTEP) {
        rowc[buf * 2 * QSTEP + tid] = rl;
        rowc[buf * 2 * QSTEP + QSTEP + tid] = rd;
      }
    };
    load_rows(qt_begin, 0);
    store_rows(0);
    mw_cur = mw_next;
    __syncthreads();
    ATTN_STAMP(1);

    // Tile qt_begin holds every diagonal sub-tile of the item (masked kind, fully
    // masked sub-tiles skipped); later full tiles are straight-line unmasked; a ragged
    // last tile (S % 64) is masked again.
    auto step = [&](auto maskc, int t) {
      constexpr bool MASKED = decltype(maskc)::value;
      const int cur = (t - qt_begin) & 1;
      const bool more = t + 1 < nqt;
      const uint32_t mw0 = mw_cur.x, mw1 = mw_cur.y;
      if (more) load_rows(t + 1, cur ^ 1);
      const bf16_t* Qt = lds + cur * 2 * QSTEP * D;
      const bf16_t* Dt = Qt + QSTEP * D;
      const float* rlp = rowc + cur * 2 * QSTEP;
      const float* rdp = rlp + QSTEP;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qs = t * QSTEP + 32 * qt;
        const bf16_t* Qs = Qt + 32 * qt * D;
        const bf16_t* Ds = Dt + 32 * qt * D;
        const uint32_t mw = (qt ? mw1 : mw0) >> (4 * h);
        if (!MASKED)
          dkdv_subtile<false, DROP, HK, D>(dka, dva, Qs, Ds, rlp + 32 * qt, rdp + 32 * qt, mw, kf, vf, qs, ka, S,
                                           lane, c_log2, dscale);
        else if (qs + 31 >= k0)
          dkdv_subtile<true, DROP, HK, D>(dka, dva, Qs, Ds, rlp + 32 * qt, rdp + 32 * qt, mw, kf, vf, qs, ka, S,
                                          lane, c_log2, dscale);
      }
      if (more) store_rows(cur ^ 1);
      mw_cur = mw_next;
      tile_barrier();
    };
    int t = qt_begin;
    const int t_full = S / QSTEP;
    if (t < nqt) step(MSK{}, t++);
    ATTN_STAMP(2);
    for (; t < t_full; ++t) step(UNM{}, t);
    for (; t < nqt; ++t) step(MSK{}, t);
    ATTN_STAMP(3);

    if (ka < S) {
      store_head_row<HK, D>(dk + hout + (size_t)ka * out_rs, dka, DROP ? scale * dscale : scale, h, cosT, sinT, ka);
      store_head_row<HK, D>(dv + hout + (size_t)ka * out_rs, dva, DROP ? dscale : 1.f, h, nullptr, nullptr, 0);
    }
#ifdef DLT_ATTN_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ATTN_STAMP(4);
    if (lane == 0) g_attn_tim[((size_t)blockIdx.x * 2 + wid) * 8 + 5] = (unsigned long long)(nqt - qt_begin);
#endif
  }
}

// ---------------------------------------------------------------------- dQ
template <bool MASK, bool DROP, int HK, int D>
__device__ __forceinline__ void dq_tile(floatx16_t (&dqa)[D / 32], const bf16_t* Kt, const bf16_t* Vt,
                                        const bf16x8_t (&qf)[D / 16], const bf16x8_t (&df)[D / 16], int k0, int qa,
                                        int S, int lane, float c_log2, float nl2, float dl, float dscale, uint2 mw) {
  constexpr int NS = D / 16;
  const int h = lane >> 5, ql = lane & 31;
  floatx16_t sacc[2], pacc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    sacc[t] = zero16();
    pacc[t] = zero16();
#if DLT_ATTN_KREAD_ASM
    // the half-tile's K and V fragments in flight at once, one counted wait each
    bf16x8_t kf[NS], vf[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) kf[s] = lds_row8_asm<D>(Kt, 32 * t + ql, 16 * s + 8 * h);
#pragma unroll
    for (int s = 0; s < NS; ++s) vf[s] = lds_row8_asm<D>(Vt, 32 * t + ql, 16 * s + 8 * h);
    if constexpr (D == 64) {
      lgkm_wait4(kf[0], kf[1], kf[2], kf[3]);
    } else {
      lgkm_wait8(kf[0], kf[1], kf[2], kf[3]);
      pin4(kf[4], kf[5], kf[6], kf[7]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) sacc[t] = mfma<HK>(kf[s], qf[s], sacc[t]);
    tr_wait_all(vf);
#pragma unroll
    for (int s = 0; s < NS; ++s) pacc[t] = mfma<HK>(vf[s], df[s], pacc[t]);
#else
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      sacc[t] = mfma<HK>(lds_row8<D>(Kt, 32 * t + ql, 16 * s + 8 * h), qf[s], sacc[t]);
      pacc[t] = mfma<HK>(lds_row8<D>(Vt, 32 * t + ql, 16 * s + 8 * h), df[s], pacc[t]);
    }
#endif
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint32_t word = DROP ? ((t ? mw.y : mw.x) >> (4 * h)) : 0u;  // prefetched a tile ahead
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kr = acc_row(i, h);
      float p = fast_exp2(fmaf(sacc[t][i], c_log2, nl2));
      if (MASK) {
        const int kA = k0 + 32 * t + kr;
        p = (kA > qa || kA >= S) ? 0.f : p;
      }
      float dp = pacc[t][i];
      if (DROP) {
        dp = keep_and(dp, keep_ones(word, (i & 3) + 8 * (i >> 2)));
        pacc[t][i] = p * fmaf(dp, dscale, -dl);
      } else {
        pacc[t][i] = p * (dp - dl);
      }
    }
  }
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const bf16x8_t sb = acc_frag<HK>(pacc[kk >> 1], kk & 1);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) dqa[dt] = mfma<HK>(tr_frag<D>(Kt, kk, dt, lane), sb, dqa[dt]);
  }
}

template <bool DROP, int HK, int D>
__global__ __launch_bounds__(NT) ATTN_WAVES(D) void k_attn_bwd_dq(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                       const bf16_t* __restrict__ v, const bf16_t* __restrict__ dout,
                                                       const bf16_t* __restrict__ o,
                                                       const float* __restrict__ lse,
                                                       float* __restrict__ delta,
                                                       const uint32_t* __restrict__ mask, bf16_t* __restrict__ dq,
                                                       int S, int nh, float c_log2, float scale, float dscale,
                                                       long in_bs, int in_hs, int in_rs, long out_bs, int out_hs,
                                                       int out_rs, const float* __restrict__ cosT,
                                                       const float* __restrict__ sinT, int xcd_map) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * KVB * D];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, ql = lane & 31;
  const int nrb = (S + RB - 1) / RB;
  int bh, pair;
  const bool lpt = work_item(nrb, xcd_map, bh, pair);
  const int b = bh / nh, head = bh % nh;
  const size_t hin = (size_t)b * in_bs + (size_t)head * in_hs;     // q / k / v
  const size_t hout = (size_t)b * out_bs + (size_t)head * out_hs;  // dq
  const int W = (S + 31) >> 5;
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using UNM = std::integral_constant<bool, false>;
  using MSK = std::integral_constant<bool, true>;

#pragma unroll 1
  for (int it = 0; it < 2; ++it) {
    const int qb = (lpt || it == 0) ? nrb - 1 - pair : pair;  // long item first
    if (it == 1 && (lpt || qb >= nrb - 1 - pair)) break;
    const int q0 = qb * RB + wid * 32;
    const int qa = q0 + ql;
    const bool qok = qa < S;
    const int qc = min(qa, S - 1);
    const uint32_t* mrow = mask ? mask + (size_t)bh * W * S + qc : nullptr;  // word j at mrow[j*S]

    bf16x8_t qf[D / 16], df[D / 16];
    const size_t orow = (((size_t)b * S + qc) * nh + head) * D;
    float dsum = 0.f;  // Delta = rowsum(dO * O), computed here (this kernel runs before dK/dV)
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      qf[s] = load_row8(q + hin + (size_t)qc * in_rs + 16 * s + 8 * h, qok);
      df[s] = load_row8(dout + orow + 16 * s + 8 * h, qok);
      const bf16x8_t of = load_row8(o + orow + 16 * s + 8 * h, qok);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += frag_f<HK>(df[s], j) * frag_f<HK>(of, j);
    }
    const float nl2 = qok ? -lse[(size_t)bh * S + qc] * LOG2E : 0.f;
    const float dl = xhalf_sum(dsum);
    if (qok && h == 0) delta[(size_t)bh * S + qa] = dl;
    floatx16_t dqa[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) dqa[dt] = zero16();

    const int nkv = (min(S, qb * RB + RB) + KVB - 1) / KVB;
    glds_tile<D>(k + hin, 0, S, in_rs, lds, wid, lane);
    glds_tile<D>(v + hin, 0, S, in_rs, lds + KVB * D, wid, lane);
    __syncthreads();

    // Same loop structure as the forward: straight-line unmasked tiles (static LDS
    // buffers, unrolled by two), then the diagonal tile.
    uint2 mw_cur = make_uint2(0u, 0u), mw_next = make_uint2(0u, 0u);
    if (DROP) mw_cur = make_uint2(mrow[0], W > 1 ? mrow[S] : 0u);
    auto step = [&](auto bufc, auto maskc, int kb) {
      constexpr int BUF = decltype(bufc)::value;
      constexpr bool MASKED = decltype(maskc)::value;
      const bool more = kb + 1 < nkv;
      if (more) {  // next tile straight into the other buffer (read by nobody since the last barrier)
        bf16_t* Kn = lds + (BUF ^ 1) * 2 * KVB * D;
        glds_tile<D>(k + hin, (kb + 1) * KVB, S, in_rs, Kn, wid, lane);
        glds_tile<D>(v + hin, (kb + 1) * KVB, S, in_rs, Kn + KVB * D, wid, lane);
        if (DROP) mw_next = make_uint2(mrow[(size_t)(2 * (kb + 1)) * S], 2 * (kb + 1) + 1 < W ? mrow[(size_t)(2 * (kb + 1) + 1) * S] : 0u);
      }
      const bf16_t* Kt = lds + BUF * 2 * KVB * D;
      const bf16_t* Vt = Kt + KVB * D;
      const int k0 = kb * KVB;
      if (!MASKED)
        dq_tile<false, DROP, HK, D>(dqa, Kt, Vt, qf, df, k0, qa, S, lane, c_log2, nl2, dl, dscale, mw_cur);
      else if (k0 <= q0 + 31)
        dq_tile<true, DROP, HK, D>(dqa, Kt, Vt, qf, df, k0, qa, S, lane, c_log2, nl2, dl, dscale, mw_cur);
      mw_cur = mw_next;
      tile_barrier();
    };
    const int nfull = min(qb, nkv);
    int kb = 0;
    for (; kb + 1 < nfull; kb += 2) {
      step(B0{}, UNM{}, kb);
      step(B1{}, UNM{}, kb + 1);
    }
    if (kb < nfull) {
      step(B0{}, UNM{}, kb);
      if (kb + 1 < nkv) step(B1{}, MSK{}, kb + 1);
    } else if (kb < nkv) {
      step(B0{}, MSK{}, kb);
    }
    if (qok) store_head_row<HK, D>(dq + hout + (size_t)qa * out_rs, dqa, scale, h, cosT, sinT, qa);
  }
}

// ============================================================================ launchers
#include <cstdlib>
// head_dim dispatch: HDC = 64 or 128 inside the body
#define DLT_HD_DISPATCH(hd, ...) \
  do {                           \
    if ((hd) == 128) {           \
      constexpr int HDC = 128;   \
      __VA_ARGS__;               \
    } else {                     \
      constexpr int HDC = 64;    \
      __VA_ARGS__;               \
    }                            \
  } while (0)
static inline bool attn_hd_ok(int hd) { return hd == 64 || hd == 128; }
// XCD-aware work map on by default; DLT_ATTN_XCD=0 restores the natural order (A/B).
static int xcd_map_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DLT_ATTN_XCD");
    v = (e && atoi(e) == 0) ? 0 : 1;
    // default: one item per workgroup, longest first (see work_item; measured B8 nh12
    // S1024: fwd 63 -> 60 us incl. the keep bits, bwd 108 -> 96 us; B16: 117 -> 105,
    // 218 -> 197); DLT_ATTN_SCHED=pair restores the paired items
    const char* sch = getenv("DLT_ATTN_SCHED");
    if (!(sch && sch[0] == 'p')) v |= 2;
  }
  return v;
}
// grid of the MFMA kernels for a work schedule
static inline int attn_grid(int nrb, int BH, int sched) { return (sched & 2) ? nrb * BH : ((nrb + 1) / 2) * BH; }
// mask: uint32 [2][B*nh, ceil(S/32), S] keep-bits written by the forward when dropout
// is on -- [0] row layout (lane = query), [1] transposed (lane = key), see
// k_dropout_bits.
// Keep-bit masks only (they depend on the key, not on the data): lets the engine
// produce them on a side stream ahead of the layer's GEMMs.
DLT_API int dlt_attn_dropout_mask(uint32_t* mask, int B, int nh, int S, uint32_t key, uint32_t thr,
                                  hipStream_t st) {
  if (S <= 0 || !mask || !thr) return -1;
  const int W = (S + 31) / 32;
  const int ntiles = W * (W + 1) / 2;  // 8 tiles (2 per wave) per block
  uint32_t* maskT = mask + (size_t)B * nh * S * W;
  k_dropout_bits<<<dim3((ntiles + 7) / 8, B * nh), 256, 0, st>>>(mask, maskT, B * nh, S, key, thr);
  DLT_CHECK_LAUNCH();
}

// gen_mask = 0: the keep bits are already in `mask` (dlt_attn_dropout_mask).
// q/k/v element (b, head, row, d) lives at base + b*in_bs + head*in_hs + row*in_rs + d:
// head-major [B*nh, S, 64] (bs = nh*S*64, hs = S*64, rs = 64) or straight inside the
// packed [B*S, 3H] QKV GEMM output (bs = S*3H, hs = 64, rs = 3H; k, v = q + H, q + 2H).
DLT_API int dlt_attn_fwd_ex(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, uint32_t* mask,
                            int B, int nh, int S, int hd, float scale, uint32_t key, uint32_t thr, float dscale,
                            int gen_mask, long in_bs, int in_hs, int in_rs, int hk, hipStream_t st) {
  if (!attn_hd_ok(hd) || S <= 0 || in_rs % 8 || in_hs % 8 || in_bs % 8) return -1;
  if (thr && !mask) return -2;  // dropout needs the keep-bit buffer
  const int nrb = (S + RB - 1) / RB;
  const int xm = xcd_map_enabled();
  const dim3 grid(attn_grid(nrb, B * nh, xm));  // work items, see work_item()
  const float c_log2 = scale * LOG2E;
  if (thr) {
    if (gen_mask) {
      const int rc = dlt_attn_dropout_mask(mask, B, nh, S, key, thr, st);
      if (rc) return rc;
    }
    DLT_HD_DISPATCH(hd, DLT_HK_DISPATCH(hk, k_attn_fwd<true, HKC, HDC><<<grid, NT, 0, st>>>(
                                                q, k, v, o, lse, mask, S, nh, c_log2, dscale, in_bs, in_hs, in_rs, xm)));
  } else {
    DLT_HD_DISPATCH(hd, DLT_HK_DISPATCH(hk, k_attn_fwd<false, HKC, HDC><<<grid, NT, 0, st>>>(
                                                q, k, v, o, lse, nullptr, S, nh, c_log2, dscale, in_bs, in_hs, in_rs, xm)));
  }
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, uint32_t* mask,
                         int B, int nh, int S, int hd, float scale, uint32_t key, uint32_t thr, float dscale,
                         int gen_mask, int hk, hipStream_t st) {
  return dlt_attn_fwd_ex(q, k, v, o, lse, mask, B, nh, S, hd, scale, key, thr, dscale, gen_mask,
                         (long)nh * S * hd, S * hd, hd, hk, st);
}

// dq/dk/dv use the (out_bs, out_hs, out_rs) layout; with cosT/sinT ([>= S, 32] fp32)
// the inverse RoPE rotation is applied to dq and dk in the store (the gradient w.r.t.
// the pre-rotation q/k of the packed QKV).
DLT_API int dlt_attn_bwd_ex(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                            const float* lse, const uint32_t* mask, float* delta_ws, bf16_t* dq, bf16_t* dk,
                            bf16_t* dv, int B, int nh, int S, int hd, float scale, float dscale, long in_bs,
                            int in_hs, int in_rs, long out_bs, int out_hs, int out_rs, const float* cosT,
                            const float* sinT, int hk, hipStream_t st) {
  if (!attn_hd_ok(hd) || S <= 0 || in_rs % 8 || in_hs % 8 || in_bs % 8 || out_rs % 4 || out_hs % 4 || out_bs % 4)
    return -1;
  if ((cosT == nullptr) != (sinT == nullptr)) return -3;
  const float c_log2 = scale * LOG2E;
  const int nrb = (S + RB - 1) / RB;
  const int xm = xcd_map_enabled();
  const dim3 gk(attn_grid(nrb, B * nh, xm)), gq(attn_grid(nrb, B * nh, xm));  // work items, see work_item()
  // dQ first: it also produces Delta = rowsum(dO * O) (no separate kernel), which
  // dK/dV then reads.
  if (mask) {
    const uint32_t* maskT = mask + (size_t)B * nh * S * ((S + 31) / 32);
    DLT_HD_DISPATCH(hd, DLT_HK_DISPATCH(hk, k_attn_bwd_dq<true, HKC, HDC><<<gq, NT, 0, st>>>(
                            q, k, v, dout, o, lse, delta_ws, mask, dq, S, nh, c_log2, scale, dscale, in_bs, in_hs,
                            in_rs, out_bs, out_hs, out_rs, cosT, sinT, xm)));
    DLT_HD_DISPATCH(hd, DLT_HK_DISPATCH(hk, k_attn_bwd_dkdv<true, HKC, HDC><<<gk, NT, 0, st>>>(
                            q, k, v, dout, lse, delta_ws, maskT, dk, dv, S, nh, c_log2, scale, dscale, in_bs, in_hs,
                            in_rs, out_bs, out_hs, out_rs, cosT, sinT, xm)));
  } else {
    DLT_HD_DISPATCH(hd, DLT_HK_DISPATCH(hk, k_attn_bwd_dq<false, HKC, HDC><<<gq, NT, 0, st>>>(
                            q, k, v, dout, o, lse, delta_ws, mask, dq, S, nh, c_log2, scale, dscale, in_bs, in_hs,
                            in_rs, out_bs, out_hs, out_rs, cosT, sinT, xm)));
    DLT_HD_DISPATCH(hd, DLT_HK_DISPATCH(hk, k_attn_bwd_dkdv<false, HKC, HDC><<<gk, NT, 0, st>>>(
                            q, k, v, dout, lse, delta_ws, mask, dk, dv, S, nh, c_log2, scale, dscale, in_bs, in_hs,
                            in_rs, out_bs, out_hs, out_rs, cosT, sinT, xm)));
  }
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                         const float* lse, const uint32_t* mask, float* delta_ws, bf16_t* dq, bf16_t* dk, bf16_t* dv,
                         int B, int nh, int S, int hd, float scale, float dscale, int hk, hipStream_t st) {
  const long bs = (long)nh * S * hd;
  return dlt_attn_bwd_ex(q, k, v, o, dout, lse, mask, delta_ws, dq, dk, dv, B, nh, S, hd, scale, dscale, bs, S * hd,
                         hd, bs, S * hd, hd, nullptr, nullptr, hk, st);
}
