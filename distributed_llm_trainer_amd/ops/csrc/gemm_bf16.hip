// Persistent bf16 "TN" GEMM for the transformer projections (gfx950 / MI355X):
//   C[M,N] = A[M,K] . B[N,K]^T      (both operands K-contiguous, fp32 accumulate)
// with fused epilogues (plain store, RoPE on q/k, SwiGLU) -- the forward GEMMs of
// /root/reference/src/models/gpt.py:185-196 (q/k/v + RoPE), :278-280 (gate/up + SwiGLU),
// :239 (o) and :281 (down), each packed into one GEMM.
//
// Why a new kernel (round 3): the projections have K = 768 (12 K-tiles), so a
// one-tile-per-workgroup GEMM spends most of its time in the prologue (first two K-tiles
// in flight, nothing to compute) and the epilogue (C stores, nothing to overlap).  This
// kernel is PERSISTENT: a workgroup walks tiles b, b + G, ... and its LDS-DMA producer
// runs straight on into the next tile's K-tiles while the current tile's last phases
// compute, so the next tile's prologue is already in flight when the epilogue stores
// are issued (the stores count in vmcnt but are younger than the prefetched K-tiles, so
// the counted waits of the next tile never wait for them).
//
// Tile BM = 256 x BN (BN = 192: N = 768 / 2304 / 3072 / 6144 / 50304 give whole rounds
// of 256 tiles at M = 16384; the template also takes 256), BK = 64, 512 threads = 8 waves as 4 (M) x 2 (N):
// each wave owns 64 x BN/2 outputs = 4 x NT tiles of v_mfma_f32_16x16x32_bf16.
// Each K-tile is consumed in 4 quadrant phases (2 m-tiles x NT/2 n-tiles x 2 k-steps):
//   q0 = (m-half 0, n-half 0): reads A-unit 0, B n-tiles 0..NT/2-1
//   q1 = (m-half 0, n-half 1): reads B n-tiles NT/2..NT-1
//   q2 = (m-half 1, n-half 1): reads A-unit 1
//   q3 = (m-half 1, n-half 0): registers only
// Staging units (LDS-DMA, source-side XOR swizzle, conflict-free ds_read_b128):
//   A0/A1 = the 32-row halves of every wave's 64 rows (128 rows, 2 DMA per wave),
//   B0 = n-tiles 0..3 of both N halves (128 rows, 2 DMA), B1 = the rest (BN-128 rows).
// Schedule (cdna_hip_programming.md §5 8-phase template): one unit per phase, restaged
// >= 2 phases after its last read (WAR), each buffer retired by a COUNTED vmcnt(4) one
// phase before it is read (RAW), raw s_barrier only; waves 4-7 run one barrier behind
// waves 0-3 so every SIMD pairs one wave's MFMA segment with its partner's LDS/DMA
// segment; MFMA clusters at s_setprio(1).
//
// Output layout: swapped product D = B_tile . A_tile^T, so a lane owns one output row
// and 4 consecutive columns per 16x16 tile; one v_permlane16_swap per packed dword pair
// regroups two neighbouring n-tiles into 8 consecutive columns -> 16-byte stores.
//
// Requirements (launcher-checked): M % 256 == 0, N % BN == 0, K % 128 == 0, rows
// 16-byte aligned.
#include "common.h"
#include "gemm_common.h"

#include <type_traits>

typedef __attribute__((address_space(3))) void* gb_lds_vptr_t;
typedef const __attribute__((address_space(1))) void* gb_gbl_cvptr_t;

namespace {

constexpr int GB_BM = 256;
constexpr int GB_BK = 64;
// LDS-transposed C stores (flags & 1024): per wave one 16-row x 96-column staging block,
// rows padded to 104 elements (52 dwords: the 8-row lane groups of the ds_write_b128
// land on disjoint banks)
constexpr int GB_STG_ROW = 104;
constexpr int GB_STG = 8 * 16 * GB_STG_ROW;
// SWIGLU: s is staged in its own per-wave 16 x 48 block (rows padded to 56 elements)
constexpr int GB_SSTG_ROW = 56;
constexpr int GB_SSTG = 8 * 16 * GB_SSTG_ROW;

__device__ __forceinline__ int gb_swz(int row, int chunk) { return row * GB_BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

template <int BN>
struct GbCfg {
  static constexpr int NT = BN / 32;           // 16-col n-tiles per wave
  static constexpr int NH = NT / 2;            // n-tiles per quadrant
  static constexpr int B1_DMA = (BN - 128) / 64;  // DMA instructions per wave for unit B1
  static constexpr int IMG_A = GB_BM * GB_BK;  // elements
  static constexpr int IMG_B = BN * GB_BK;
  static constexpr int BUF = IMG_A + IMG_B;
};

// Tile row of the first row of 8-row group g of a staging unit.
//   A unit q: rows {wm*64 + q*32 + 0..31 : wm = 0..3}
//   B unit 0: rows {wn*BN/2 + 0..63 : wn = 0..1}; unit 1: rows {wn*BN/2 + 64 .. BN/2-1}
template <int BN>
__device__ __forceinline__ int gb_arow(int q, int g) { return (g >> 2) * 64 + q * 32 + (g & 3) * 8; }
template <int BN>
__device__ __forceinline__ int gb_brow(int q, int g) {
  if (q == 0) return (g >> 3) * (BN / 2) + (g & 7) * 8;
  constexpr int per = (BN / 2 - 64) / 8;  // groups per N half in unit 1 (none at BN = 128)
  if constexpr (per == 0) return 0;
  else return (g / per) * (BN / 2) + 64 + (g % per) * 8;
}

}  // namespace

// Epilogues.  ROPE and SWIGLU (BN = 192 only) permute the B rows of a tile so that the
// two operands of each element-pair op land in the SAME lane: wave-local n-tile t < 3
// and t + 3 hold, for ROPE, head dims j and j + 32 of the same 16-pair block (the tile
// covers 3 heads = 96 rotation pairs, 48 per wave); for SWIGLU, gate and up rows of the
// same 16 intermediate indices (the tile covers 96 intermediate indices, so the tile
// stride in W rows is 96).  The stores use the same map, so C keeps its natural layout.
//   STORE : C = A.B^T
//   ROPE  : C = A.Wqkv^T with NeoX RoPE on the q and k heads (columns < rot_cols) at
//           position row % S -- the reference's q/k/v projections + apply_rotary_pos_emb
//           (gpt.py:185-196) in one pass; same math as k_rope_qk_inplace on the bf16
//           GEMM output (elementwise.hip).
//   SWIGLU: gu = A.Wgu^T (gate | up, [M, 2I]) and s = silu(g) * u ([M, I]) -- gpt.py:278-280;
//           same math as k_swiglu_fwd on the bf16 gate/up values.
//   SWIGLU_BWD (data-gradient form, BT): ds = dd . Wdown (the down projection's input
//           gradient, [M, I]) and, per element, the SwiGLU backward of gpt.py:280 on the
//           kept gu = [gate | up] (same math as k_swiglu_bwd on the bf16-rounded ds):
//           dgu[:, j] = ds * u * sig(g) * (1 + g (1 - sig(g))), dgu[:, I + j] = ds * silu(g).
enum { GB_EPI_STORE = 0, GB_EPI_ROPE = 1, GB_EPI_SWIGLU = 2, GB_EPI_SWIGLU_BWD = 3 };

// Diagnostic build only (tools/cpp/gemm_bench.cpp defines GB_STAMPS): per-wave s_memtime
// sums of the first K-iteration of a tile, the rest of its K-loop and its epilogue, plus
// the kernel's shader-clock / real-time span, written by lane 0 to gb_stamp_buf.
#ifdef GB_STAMPS
__device__ unsigned long long* gb_stamp_buf;
#define GB_T() __builtin_amdgcn_s_memtime()
#endif

struct GbEpi {
  const float* cosT;  // ROPE: [S_tab, 32] fp32
  const float* sinT;
  int S;              // ROPE: sequence length (position = row % S)
  int rot_cols;       // ROPE: columns [0, rot_cols) are rotated (2H: q and k)
  bf16_t* s_out;      // SWIGLU: s [M, ld_s]
  int ld_s;
  int I;              // SWIGLU: intermediate size (gate rows [0, I), up rows [I, 2I))
  const bf16_t* gu_in;  // SWIGLU_BWD: kept gu [M, 2I] (row stride ld_s)
};

// Column (== B row) offset of wave-local n-tile t's first column within its tile.
template <int BN, int EPI>
__device__ __forceinline__ int gb_ncol(int wn, int t, int I) {
  if constexpr (EPI == GB_EPI_STORE || EPI == GB_EPI_SWIGLU_BWD) {
    return wn * (BN / 2) + t * 16;
  } else {
    const int P = wn * 48 + (t % 3) * 16;  // rotation pair / intermediate index
    if constexpr (EPI == GB_EPI_ROPE)
      return (P >> 5) * 64 + (P & 31) + (t >= 3 ? 32 : 0);
    else
      return P + (t >= 3 ? I : 0);
  }
}
// tile-local B row r (0..BN-1) -> row of B relative to the tile's base row
template <int BN, int EPI>
__device__ __forceinline__ int gb_bmap(int r, int I) {
  return gb_ncol<BN, EPI>(r / (BN / 2), (r % (BN / 2)) >> 4, I) + (r & 15);
}

// One 16-byte-per-lane LDS-DMA piece issued from inline asm: the compiler's wait pass does
// not see it.  For an LDS-DMA it knows about, that pass waits vmcnt(0) before the first use
// of ANY older load's result (it does not count LDS-DMA in order with the loads), which
// turned the epilogue-first staging's gu / cos-sin waits into waits for the whole next-tile
// prefetch.  Invisible pieces only ever make the compiler's counted waits stricter (it
// counts fewer younger operations than are in flight), never unsafe; the code that reads
// the staged LDS waits for them with its own counted s_waitcnt.
__device__ __forceinline__ void gb_dma_asm(const void* g, const void* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

// 4 fp32 -> 4 bf16 (RNE) as two v_cvt_pk_bf16_f32; and back (exact)
typedef __bf16 gb_bf16x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t gb_u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 gb_pack(const floatx4_t& v) {
  return __builtin_bit_cast(uint2, __builtin_convertvector(v, gb_bf16x4_t));
}
// the plain store epilogue's pack for IEEE-half output (HK = 1, --mixed_precision fp16)
typedef _Float16 gb_f16x4_t __attribute__((ext_vector_type(4)));
template <int HK>
__device__ __forceinline__ uint2 gb_pack_hk(const floatx4_t& v) {
  if constexpr (HK == 0) return gb_pack(v);
  else return __builtin_bit_cast(uint2, __builtin_convertvector(v, gb_f16x4_t));
}
// two 16-bit values of one dword (low half first) as floats, in the operand format
template <int HK>
__device__ __forceinline__ void gb_unpack2(uint32_t w, float (&f)[2]) {
  if constexpr (HK == 0) {
    f[0] = __uint_as_float(w << 16);
    f[1] = __uint_as_float(w & 0xffff0000u);
  } else {
    f[0] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
    f[1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
  }
}
__device__ __forceinline__ void gb_unpack(uint2 p, float (&f)[4]) {
  f[0] = __uint_as_float(p.x << 16);
  f[1] = __uint_as_float(p.x & 0xffff0000u);
  f[2] = __uint_as_float(p.y << 16);
  f[3] = __uint_as_float(p.y & 0xffff0000u);
}

// BT = false: C = A . B^T with B[N, K] (the forward projections, K contiguous in both).
// BT = true (data gradients): C = A . B with B[K, N] read AS STORED -- dX = dY . W for a
// weight W[Nred, Nout] -- the B staging units become reduction-major images (B0: 64
// reduction rows x 128 columns = n-tiles 0..3 of both N halves, B1: 64 x 64 = n-tiles
// 4..5), filled by LDS-DMA of whole 256 / 128-byte row pieces with a per-row XOR chunk
// swizzle and read with ds_read_b64_tr_b16 (gemm_common.h, as k_gemm_wgrad reads its
// token-major operands).  Same unit sizes and DMA counts per wave, so the 8-phase
// schedule and its counted waits are unchanged.
// HK: operand / output format, 0 = bf16, 1 = IEEE half (plain store epilogue only).
// LATE (ROPE / SWIGLU_BWD only): epilogue-first staging of the next tile, see the loop.
template <int BN, int EPI, bool BT = false, int HK = 0, bool LATE = false>
__global__ __launch_bounds__(512, 1) void k_gemm_bf16(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                      bf16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                      int ldc, int flags, GbEpi ep) {
  static_assert(EPI == GB_EPI_STORE || BN == 192, "pair epilogues need the 192-column tile");
  static_assert(!BT || (BN == 192 && (EPI == GB_EPI_STORE || EPI == GB_EPI_SWIGLU_BWD)) ||
                    (BN == 128 && EPI == GB_EPI_STORE),
                "the reduction-major B form is the 192- (or plain 128-) column data-gradient kernel");
  static_assert(HK == 0 || EPI == GB_EPI_STORE || EPI == GB_EPI_SWIGLU_BWD,
                "the RoPE / SwiGLU forward epilogues are bf16-only");
  static_assert(!LATE || EPI == GB_EPI_ROPE || EPI == GB_EPI_SWIGLU_BWD, "epilogue-first staging: loading epilogues");
  using Cf = GbCfg<BN>;
  constexpr int TS = EPI == GB_EPI_SWIGLU ? 96 : BN;  // tile stride in B rows
  constexpr int NT = Cf::NT, NH = Cf::NH;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * Cf::BUF + GB_STG + (EPI == GB_EPI_SWIGLU ? GB_SSTG : 0)];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = wid >> 2;                  // stagger group (waves w and w+4 share a SIMD)
  const int wm = wid & 3, wn = wid >> 2;      // 4 (M) x 2 (N) wave grid
  const int l16 = lane & 15, lq = lane >> 4;

  const int ntn = N / BN;
  const int ntiles = (M / GB_BM) * ntn;
  const int G = gridDim.x;  // multiple of 8
  const int bid = blockIdx.x;
  // tile walk: round r, workgroup b on "XCD slot" x = b % 8 -> linear tile
  // r*G + x*(G/8) + b/8: the workgroups of one XCD cover G/8 consecutive tiles per round
  const int gx = G >> 3;
  // order 3 (flags bits 2-3): XCD row bands -- XCD slot x owns tile rows
  // [x * ntm/8, (x+1) * ntm/8) and walks every column tile over them (ntm/8 rows x
  // gx/(ntm/8) columns per round), so its A panels (ntm/8 x 384 KB at K = 768) stay in
  // its L2 for the whole kernel and every B panel is read once per XCD.  For the lm_head
  // (64 x 262 tiles) the grouped walk re-reads each A panel 131 times from beyond L2.
  const int ntm = M / GB_BM;
  const bool xband = ((flags >> 2) & 3) == 3 && (ntm & 7) == 0 && gx % (ntm >> 3) == 0;
  const int band = xband ? (ntm >> 3) * ntn : 0;  // tiles per XCD slot
  auto tile_of = [&](int r) {
    return xband ? (bid & 7) * band + r * gx + (bid >> 3) : r * G + (bid & 7) * gx + (bid >> 3);
  };
  const int tend = xband ? ((bid & 7) + 1) * band : ntiles;  // first tile past this workgroup's range
  // linear tile -> (tile row, tile col).  With 32 workgroups per XCD slot and whole
  // 32-tile super-tiles (GM x GN tiles, GN = 8 / 4 / 2 n-tiles), super-tile s = L / 32 is
  // one XCD's work of one round and the super-tiles walk DOWN a super-column
  // (column-major), so an XCD keeps the same GN B panels for consecutive rounds and its
  // per-round operand set (GM A panels + GN B panels, ~4 MB at K = 768) fits its L2.
  // Otherwise plain row-major.
  const int gn = (ntn & 7) == 0 ? 8 : (ntn & 3) == 0 ? 4 : (ntn & 1) == 0 ? 2 : 1;
  const int gm = 32 / gn;
  // flags (ablation only, 0 in production): bit 0 skip the C stores, bit 1 every tile
  // reads tile (0, 0)'s operand panels (L2-resident), bits 2-3 tile order (0 = grouped
  // column walk, 1 = row-major, 2 = grouped row walk, 3 = XCD row bands), 16 every tile
  // stores to tile (0, 0),
  // 32 s_waitcnt vmcnt(0) after the stores
  const int order = (flags >> 2) & 3;
  const bool grouped = order != 1 && gx == 32 && ntiles % 32 == 0 && ntm % gm == 0;
  const int scols = ntn / gn;
  const int srows = ntm / gm;
  auto coords = [&](int L, int& tm, int& tn) {
    if (xband) {
      const int rpx = ntm >> 3, x = L / band, j = L - x * band;
      tm = x * rpx + j % rpx;
      tn = j / rpx;
    } else if (grouped) {
      const int sidx = L >> 5, i = L & 31;
      if (order == 2) {
        tm = (sidx / scols) * gm + i / gn;
        tn = (sidx % scols) * gn + i % gn;
      } else {
        tm = (sidx % srows) * gm + i / gn;
        tn = (sidx / srows) * gn + i % gn;
      }
    } else {
      tm = L / ntn;
      tn = L % ntn;
    }
  };

  bf16_t* const A0i = lds;
  bf16_t* const B0i = lds + Cf::IMG_A;
  bf16_t* const A1i = lds + Cf::BUF;
  bf16_t* const B1i = lds + Cf::BUF + Cf::IMG_A;

  // per-lane source offsets (bytes, relative to the tile's first row at column kt*BK)
  uint32_t oa[2][2], ob0[2], ob1[Cf::B1_DMA > 0 ? Cf::B1_DMA : 1];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = gb_arow<BN>(q, wid * 2 + j) + (lane >> 3);
      oa[q][j] = (uint32_t)(row * lda + (((lane & 7) ^ ((row >> 1) & 7)) << 3)) * 2u;
    }
  // (the swizzle follows the LDS image row; the source row goes through the epilogue's
  // B-row map)
  if constexpr (BT) {
    // reduction-major B: DMA piece e of unit B0 = 16-byte chunk pc of reduction row t
    // (16 chunks per 256-byte image row), source chunk lc = pc ^ 2 v(t) (gemm_common.h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = (wid * 2 + j) * 64 + lane;
      const int t = e >> 4, lc = (e & 15) ^ (2 * gw_v256(t));
      ob0[j] = (uint32_t)(t * ldb + gw_b0map<BN>(lc * 8)) * 2u;
    }
    if constexpr (Cf::B1_DMA > 0) {
      const int e = wid * 64 + lane;
      const int t = e >> 3, lc = (e & 7) ^ (2 * gw_v128(t));
      ob1[0] = (uint32_t)(t * ldb + gw_b1map(lc * 8)) * 2u;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = gb_brow<BN>(0, wid * 2 + j) + (lane >> 3);
      ob0[j] = (uint32_t)(gb_bmap<BN, EPI>(row, ep.I) * ldb + (((lane & 7) ^ ((row >> 1) & 7)) << 3)) * 2u;
    }
#pragma unroll
    for (int j = 0; j < Cf::B1_DMA; ++j) {
      const int row = gb_brow<BN>(1, wid * Cf::B1_DMA + j) + (lane >> 3);
      ob1[j] = (uint32_t)(gb_bmap<BN, EPI>(row, ep.I) * ldb + (((lane & 7) ^ ((row >> 1) & 7)) << 3)) * 2u;
    }
  }

  // (LATE kernels: every piece from inline asm, gb_dma_asm -- with any compiler-visible
  // LDS-DMA possibly in flight at the K-loop exit, the compiler made the epilogue's first
  // load use wait vmcnt(0); the K-loop's own counted waits + barriers are what orders
  // the LDS images, in every variant)
  auto stA = [&](const bf16_t* g, int q, bf16_t* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (LATE)
        gb_dma_asm((const char*)g + oa[q][j], img + gb_arow<BN>(q, wid * 2 + j) * GB_BK);
      else
        __builtin_amdgcn_global_load_lds((gb_gbl_cvptr_t)((const char*)g + oa[q][j]),
                                         (gb_lds_vptr_t)(img + gb_arow<BN>(q, wid * 2 + j) * GB_BK), 16, 0, 0);
    }
  };
  auto stB0 = [&](const bf16_t* g, bf16_t* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16_t* dst = img + (BT ? (wid * 2 + j) * 512 : gb_brow<BN>(0, wid * 2 + j) * GB_BK);
      if constexpr (LATE)
        gb_dma_asm((const char*)g + ob0[j], dst);
      else
        __builtin_amdgcn_global_load_lds((gb_gbl_cvptr_t)((const char*)g + ob0[j]), (gb_lds_vptr_t)dst, 16, 0, 0);
    }
  };
  // the same units from inline asm (LATE staging: gb_dma_asm)
  auto stA_asm = [&](const bf16_t* g, int q, bf16_t* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      gb_dma_asm((const char*)g + oa[q][j], img + gb_arow<BN>(q, wid * 2 + j) * GB_BK);
  };
  auto stB0_asm = [&](const bf16_t* g, bf16_t* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      gb_dma_asm((const char*)g + ob0[j], img + (BT ? (wid * 2 + j) * 512 : gb_brow<BN>(0, wid * 2 + j) * GB_BK));
  };
  auto stB1_asm = [&](const bf16_t* g, bf16_t* img) {
#pragma unroll
    for (int j = 0; j < Cf::B1_DMA; ++j)
      gb_dma_asm((const char*)g + ob1[j],
                 img + (BT ? GW_IMG_A + wid * 512 : gb_brow<BN>(1, wid * Cf::B1_DMA + j) * GB_BK));
  };
  auto stB1 = [&](const bf16_t* g, bf16_t* img) {
#pragma unroll
    for (int j = 0; j < Cf::B1_DMA; ++j) {
      bf16_t* dst = img + (BT ? GW_IMG_A + wid * 512 : gb_brow<BN>(1, wid * Cf::B1_DMA + j) * GB_BK);
      if constexpr (LATE)
        gb_dma_asm((const char*)g + ob1[j], dst);
      else
        __builtin_amdgcn_global_load_lds((gb_gbl_cvptr_t)((const char*)g + ob1[j]), (gb_lds_vptr_t)dst, 16, 0, 0);
    }
  };
  // operand pointer of K-tile kt (relative): A and the K-major B advance along the row,
  // the reduction-major B by whole rows
  auto bk = [&](const bf16_t* g, int kt) { return BT ? g + (size_t)kt * GB_BK * ldb : g + kt * GB_BK; };

  floatx4_t acc[NT][4];
  bf16x8_t fa[2][2], fb0[NH][2], fb1[NH][2];
  const int arow = wm * 64 + l16;         // + qm*32 + mt*16
  const int brow = wn * (BN / 2) + l16;   // + qn*NH*16 + nt*16
  auto read_a = [&](const bf16_t* img, int qm) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[mt][s] = *reinterpret_cast<const bf16x8_t*>(img + gb_swz(arow + qm * 32 + mt * 16, s * 4 + lq));
  };
  // BT: per-lane transposed-read bases (gemm_common.h): B0 n-tile k = 4 wn + nt, B1 k = 2 wn + j
  uint32_t kb0[4], kb1[2];
  if constexpr (BT) {
    GwLane<256> L256;
    GwLane<128> L128;
    L256.init(lane);
    L128.init(lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) kb0[j] = L256.base + L256.koff(4 * wn + j);
#pragma unroll
    for (int j = 0; j < 2; ++j) kb1[j] = L128.base + L128.koff(2 * wn + j);
  }
  auto read_b = [&](const bf16_t* img, int qn, bf16x8_t (&fb)[NH][2]) {
    if constexpr (BT && BN == 128) {
      // n-half qn: n-tiles 2qn, 2qn + 1, both from B0 (the image holds the tile's columns)
      const uint32_t i0 = (uint32_t)(uintptr_t)img;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int nt = 0; nt < NH; ++nt) fb[nt][s] = gw_frag<256>(i0 + kb0[qn * NH + nt], s);
    } else if constexpr (BT) {
      // n-half 0: n-tiles 0..2 (B0); n-half 1: n-tile 3 (B0) and 4..5 (B1)
      const uint32_t i0 = (uint32_t)(uintptr_t)img, i1 = i0 + GW_IMG_A * 2;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (qn == 0) {
#pragma unroll
          for (int nt = 0; nt < NH; ++nt) fb[nt][s] = gw_frag<256>(i0 + kb0[nt], s);
        } else {
          fb[0][s] = gw_frag<256>(i0 + kb0[3], s);
          fb[1][s] = gw_frag<128>(i1 + kb1[0], s);
          fb[2][s] = gw_frag<128>(i1 + kb1[1], s);
        }
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          fb[nt][s] = *reinterpret_cast<const bf16x8_t*>(img + gb_swz(brow + (qn * NH + nt) * 16, s * 4 + lq));
    }
  };
  auto mma = [&](int qm, int qn, bf16x8_t (&fb)[NH][2]) {
    if constexpr (BT && NH == 2) {
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                     "+v"(fb[1][0]), "+v"(fb[1][1])::"memory");
    } else if constexpr (BT) {
      // the transposed reads are asm (invisible to the compiler's lgkmcnt tracking): the
      // fragments are in/out operands of the wait so no MFMA is scheduled above it
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                     "+v"(fb[1][0]), "+v"(fb[1][1]), "+v"(fb[2][0]), "+v"(fb[2][1])::"memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
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

  const int nk = K / GB_BK;  // even, >= 2
#ifdef GB_STAMPS
  const uint64_t s_k0 = GB_T(), s_r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t a_it0 = 0, a_rest = 0, a_epi = 0, ntl = 0, t1 = 0;
#endif
  int tile = tile_of(0);
  if (tile >= tend) return;  // whole workgroup idle (uniform)
  auto abase = [&](int t) {
    int tm, tn;
    coords(t, tm, tn);
    if (flags & 2) tm = 0;
    return A + (size_t)(tm * GB_BM) * lda;
  };
  auto bbase = [&](int t) {
    int tm, tn;
    coords(t, tm, tn);
    if (flags & 2) tn = 0;
    return BT ? B + (size_t)tn * TS : B + (size_t)(tn * TS) * ldb;
  };

  // the next tile's first K-tiles, as the kernel prologue stages them (epilogue-first
  // staging, flags & 4096): K-tile 0 whole into buffer 0, A0 / B0 of K-tile 1 into buffer 1
  auto stage_next_of = [&](int t) {
    const bf16_t* Ab = abase(t);
    const bf16_t* Bb = bbase(t);
    __builtin_amdgcn_sched_barrier(0);  // the epilogue's loads stay older than these
    stA_asm(Ab, 0, A0i);
    stB0_asm(Bb, B0i);
    stB1_asm(Bb, B0i);
    stA_asm(Ab, 1, A0i);
    stA_asm(Ab + GB_BK, 0, A1i);
    stB0_asm(bk(Bb, 1), B1i);
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue: K-tile 0 of the first tile complete in buffer 0, units A0/B0 of K-tile 1
  // in flight (their steady-state slots are phases 7 and 8)
  {
    const bf16_t* Ab = abase(tile);
    const bf16_t* Bb = bbase(tile);
    stA(Ab, 0, A0i);
    stB0(Bb, B0i);
    stB1(Bb, B0i);
    stA(Ab, 1, A0i);
    stA(Ab + GB_BK, 0, A1i);
    stB0(bk(Bb, 1), B1i);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (half == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 one barrier behind
  }

  // LATE: epilogues that READ global memory (RoPE: cos/sin tables; SwiGLU backward: the
  // kept gu) issue those loads first and only then the next tile's first K-tiles
  // ("epilogue-first staging"; the launcher selects it with flags & 4096): vmcnt retires
  // in issue order, so with the next tile's DMA staged in the last K-iteration (the plain
  // epilogue's schedule) every epilogue load waited for that whole prefetch (RoPE
  // epilogue 9.3k vs 3.1k cycles, profiles/r4_gemm_forward.md section 5).  The next
  // tile's K-tile 0 then lands during the epilogue's arithmetic and stores.  Compile-time,
  // and the staging is issued on every tile (the last one re-stages its own operands,
  // never read), so the compiler's waits see one instruction count on every path (a
  // conditional staging made them vmcnt(0) at the join).
  for (int r = 0;; ++r) {
    const int next = tile_of(r + 1);
    const bool has_next = next < tend;
    const bf16_t* const Ab = abase(tile);
    const bf16_t* const Bb = bbase(tile);
    const bf16_t* const An = has_next ? abase(next) : Ab;
    const bf16_t* const Bn = has_next ? bbase(next) : Bb;
    auto stage_next = [&]() { stage_next_of(has_next ? next : tile); };
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};
#ifdef GB_STAMPS
    const uint64_t t0 = GB_T();
#endif

    for (int kt = 0; kt < nk; kt += 2) {
      // the K-tiles staged in this iteration: kt+1 (rest of it), kt+2, kt+3 -- the last
      // two belong to the next tile at the end of this one
      const bool inner = kt + 2 < nk;
      const bool more = inner || (has_next && !LATE);
      const bf16_t* const A2 = inner ? Ab + (kt + 2) * GB_BK : An;
      const bf16_t* const B2 = inner ? bk(Bb, kt + 2) : Bn;
      // ---- phase 1: buffer 0, q0 ; stage B1 of K-tile kt+1
      read_b(B0i, 0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      read_a(A0i, 0);
      stB1(bk(Bb, kt + 1), B1i);
      __builtin_amdgcn_s_barrier();
      mma(0, 0, fb0);
      __builtin_amdgcn_s_barrier();
      // ---- phase 2: q1 ; A1 of K-tile kt+1
      read_b(B0i, 1, fb1);
      stA(Ab + (kt + 1) * GB_BK, 1, A1i);
      __builtin_amdgcn_s_barrier();
      mma(0, 1, fb1);
      __builtin_amdgcn_s_barrier();
      // ---- phase 3: q2 ; A0 of K-tile kt+2 into buffer 0
      read_a(A0i, 1);
      if (more) stA(A2, 0, A0i);
      __builtin_amdgcn_s_barrier();
      mma(1, 1, fb1);
      __builtin_amdgcn_s_barrier();
      // ---- phase 4: q3 (registers) ; B0 of kt+2 ; retire K-tile kt+1
      if (more) {
        stB0(B2, B0i);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      mma(1, 0, fb0);
      __builtin_amdgcn_s_barrier();
      // ---- phase 5: buffer 1, q0 ; B1 of kt+2
      read_b(B1i, 0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      read_a(A1i, 0);
      if (more) stB1(B2, B0i);
      __builtin_amdgcn_s_barrier();
      mma(0, 0, fb0);
      __builtin_amdgcn_s_barrier();
      // ---- phase 6: q1 ; A1 of kt+2
      read_b(B1i, 1, fb1);
      if (more) stA(A2, 1, A0i);
      __builtin_amdgcn_s_barrier();
      mma(0, 1, fb1);
      __builtin_amdgcn_s_barrier();
      // ---- phase 7: q2 ; A0 of kt+3 into buffer 1
      read_a(A1i, 1);
      if (more) stA(A2 + GB_BK, 0, A1i);
      __builtin_amdgcn_s_barrier();
      mma(1, 1, fb1);
      __builtin_amdgcn_s_barrier();
      // ---- phase 8: q3 ; B0 of kt+3 ; retire K-tile kt+2
      if (more) {
        stB0(bk(B2, 1), B1i);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      mma(1, 0, fb0);
      __builtin_amdgcn_s_barrier();
#ifdef GB_STAMPS
      if (kt == 0) t1 = GB_T();
#endif
    }
#ifdef GB_STAMPS
    const uint64_t t2 = GB_T();
#endif

    // ---- epilogue: acc[nt][mt] = D[n][m]; lane owns row m0 + wm*64 + mt*16 + l16 and
    // columns (n-tile nt) + lq*4 .. +3.  permlane16_swap over n-tile pairs (2p, 2p+1):
    // lanes with lq even end up with 8 consecutive columns of n-tile 2p, lq odd of 2p+1.
    // Every f32 -> bf16 conversion is one v_cvt_pk_bf16_f32 per PAIR (gb_pack); the
    // per-element cast plus shift/or packing it replaces was ~40 % of the plain epilogue's
    // VALU, and the fused epilogues take their bf16-rounded inputs from the same packs.
    if (!(flags & 1)) {
      int tm, tn;
      coords(tile, tm, tn);
      if (flags & 16) tm = tn = 0;
      const int m0 = tm * GB_BM, n0 = tn * TS;
      if constexpr (EPI == GB_EPI_ROPE) {
        // all cos/sin loads first (the fragment registers are dead here), one wait.  The
        // lane's rotation pairs are P = wn*48 + t*16 + lq*4 + e: only two distinct
        // 4-column j blocks (t = 0 and 2 coincide mod 32)
        float4 cs[4][2], sn[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int pos = (m0 + wm * 64 + mt * 16 + l16) % ep.S;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int j = (wn * 48 + u * 16 + lq * 4) & 31;
            cs[mt][u] = *reinterpret_cast<const float4*>(ep.cosT + (size_t)pos * 32 + j);
            sn[mt][u] = *reinterpret_cast<const float4*>(ep.sinT + (size_t)pos * 32 + j);
          }
        }
        if constexpr (LATE) stage_next();
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            const int P = wn * 48 + t * 16 + lq * 4;
            if (LATE || n0 + (P >> 5) * 64 < ep.rot_cols) {
              // LATE: branch-free (cos 1 / sin 0 on the v heads) -- a branch here made the
              // compiler wait for every outstanding load, the next tile's DMA included
              const bool rot = !LATE || n0 + (P >> 5) * 64 < ep.rot_cols;
              const float4 c4 = cs[mt][t & 1], s4 = sn[mt][t & 1];
              const float cc[4] = {rot ? c4.x : 1.f, rot ? c4.y : 1.f, rot ? c4.z : 1.f, rot ? c4.w : 1.f};
              const float ss[4] = {rot ? s4.x : 0.f, rot ? s4.y : 0.f, rot ? s4.z : 0.f, rot ? s4.w : 0.f};
              float x1[4], x2[4];
              gb_unpack(gb_pack(acc[t][mt]), x1);  // the bf16 GEMM output the unfused path rotates
              gb_unpack(gb_pack(acc[t + 3][mt]), x2);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                acc[t][mt][e] = x1[e] * cc[e] - x2[e] * ss[e];
                acc[t + 3][mt][e] = x2[e] * cc[e] + x1[e] * ss[e];
              }
            }
          }
      }
      // SWIGLU_BWD: the lane's kept gate / up values for all 4 m-tiles (8 consecutive
      // columns per pair p: the same columns its permlane-swapped ds values land on)
      // Buffer loads / stores over the tile's 256 rows: ONE per-lane byte offset (row
      // l16 of the wave's first m-tile, the lane's column base) for all 24 + 24 accesses,
      // the m-tile (and the up half) in the SGPR offset, the pair p in the immediate --
      // 64-bit row pointers per access pushed the preloading kernel into spills.
      gb_u32x4_t gv[EPI == GB_EPI_SWIGLU_BWD ? 4 : 1][NT / 2], uv[EPI == GB_EPI_SWIGLU_BWD ? 4 : 1][NT / 2];
      [[maybe_unused]] __amdgpu_buffer_rsrc_t rs_gu, rs_c;
      [[maybe_unused]] int sw_voff = 0;
      if constexpr (EPI == GB_EPI_SWIGLU_BWD) {
        rs_gu = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(ep.gu_in) + (size_t)m0 * ep.ld_s, 0,
                                                  GB_BM * ep.ld_s * 2, 0x00020000);
        rs_c = __builtin_amdgcn_make_buffer_rsrc(C + (size_t)m0 * ldc, 0, GB_BM * ldc * 2, 0x00020000);
        // column of pair p: wn * 96 + (2p + (lq & 1)) * 16 + (lq >> 1) * 8 (the STORE map)
        sw_voff = ((wm * 64 + l16) * ep.ld_s + n0 + wn * (BN / 2) + (lq & 1) * 16 + (lq >> 1) * 8) * 2;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int p = 0; p < NT / 2; ++p) {
            const int so = mt * 16 * ep.ld_s * 2;
            gv[mt][p] = __builtin_bit_cast(gb_u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs_gu, sw_voff + p * 64, so, 0));
            uv[mt][p] = __builtin_bit_cast(gb_u32x4_t,
                                           __builtin_amdgcn_raw_buffer_load_b128(rs_gu, sw_voff + p * 64, so + ep.I * 2, 0));
          }
        if constexpr (LATE) stage_next();
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int row = m0 + wm * 64 + mt * 16 + l16;
        uint2 pk[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) pk[t] = gb_pack_hk<HK>(acc[t][mt]);
        // staged (LDS-transposed) stores: flag 1024; always for SWIGLU (its two stores
        // per lane otherwise write 16 rows x 32 + 8 bytes each)
        // (LATE RoPE: row-per-lane permlane stores -- the staging ds_writes would make the
        // compiler drain the next tile's in-flight LDS-DMA first)
        const bool lt = EPI == GB_EPI_SWIGLU || (EPI != GB_EPI_SWIGLU_BWD && !BT && !LATE && BN == 192 && (flags & 1024));
        if constexpr (EPI == GB_EPI_SWIGLU) {
          uint2 sp[3];
          // s = silu(g) * u on the bf16-rounded gate/up values (the packs stored as gu);
          // without the staged stores n-tiles 0/1 of s are paired for 16-byte stores and
          // n-tile 2 stores 8 bytes per lane
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            float g[4], u[4];
            gb_unpack(pk[t], g);
            gb_unpack(pk[t + 3], u);
            floatx4_t sv;
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[e] = g[e] * dlt_sigmoid(g[e]) * u[e];
            sp[t] = gb_pack(sv);
          }
          if (lt) {
            bf16_t* sstg = lds + 2 * Cf::BUF + GB_STG + wid * (16 * GB_SSTG_ROW);
#pragma unroll
            for (int t = 0; t < 3; ++t)
              *reinterpret_cast<uint2*>(sstg + l16 * GB_SSTG_ROW + t * 16 + lq * 4) = sp[t];
          } else {
            bf16_t* srow = ep.s_out + (size_t)row * ep.ld_s + (size_t)tn * 96 + wn * 48;
            uint32_t x[2] = {sp[0].x, sp[0].y}, y[2] = {sp[1].x, sp[1].y};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              auto sw = __builtin_amdgcn_permlane16_swap(x[h], y[h], false, false);
              x[h] = sw[0];
              y[h] = sw[1];
            }
            *reinterpret_cast<uint4*>(srow + (lq & 1) * 16 + (lq >> 1) * 8) = uint4{x[0], x[1], y[0], y[1]};
            *reinterpret_cast<uint2*>(srow + 32 + lq * 4) = sp[2];
          }
        }
        bf16_t* crow = C + (size_t)row * ldc + n0;
        if (lt) {
          // LDS-transposed stores: the lane's three 16-byte chunks (8 consecutive columns
          // each) go to the wave's staging block, then every store instruction writes
          // 5.33 whole row segments (12 lanes per row, consecutive lanes on consecutive
          // 16 bytes) instead of 16 rows x 64 bytes.  Staging column chunk c holds columns
          // gb_ncol(wn, c / 2) + (c % 2) * 8: one 192-byte run per row for STORE, the gate
          // and up 96-byte runs for SWIGLU, the head-pair map for ROPE.  Wave-local: the
          // wave reads back only what it wrote (LDS operations of one wave stay in order).
          bf16_t* stg = lds + 2 * Cf::BUF + wid * (16 * GB_STG_ROW);
#pragma unroll
          for (int p = 0; p < NT / 2; ++p) {
            uint32_t x[2] = {pk[2 * p].x, pk[2 * p].y}, y[2] = {pk[2 * p + 1].x, pk[2 * p + 1].y};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              auto sw = __builtin_amdgcn_permlane16_swap(x[h], y[h], false, false);
              x[h] = sw[0];
              y[h] = sw[1];
            }
            const int chunk = 4 * p + 2 * (lq & 1) + (lq >> 1);
            *reinterpret_cast<gb_u32x4_t*>(stg + l16 * GB_STG_ROW + chunk * 8) = gb_u32x4_t{x[0], x[1], y[0], y[1]};
          }
          bf16_t* cblk = C + (size_t)(m0 + wm * 64 + mt * 16) * ldc + n0;
          // write-through (sc1, flags & 2048) stores: the C lines leave the XCD's L2
          // instead of displacing the operand panels the next K-iterations read
          // (profiles/r4_gemm_forward.md section 5)
          const auto rs = __builtin_amdgcn_make_buffer_rsrc(cblk, 0, 16 * ldc * 2, 0x00020000);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const int e = i * 64 + lane, r = e / 12, c = e - r * 12;
            const int col = gb_ncol<BN, EPI>(wn, c >> 1, ep.I) + (c & 1) * 8;
            const gb_u32x4_t v = *reinterpret_cast<const gb_u32x4_t*>(stg + r * GB_STG_ROW + c * 8);
            if (flags & 2048)
              __builtin_amdgcn_raw_buffer_store_b128(v, rs, (r * ldc + col) * 2, 0, 16);
            else
              *reinterpret_cast<gb_u32x4_t*>(cblk + (size_t)r * ldc + col) = v;
          }
          if constexpr (EPI == GB_EPI_SWIGLU) {
            // s [16 rows x 48 columns] from its staging block: 96-byte row runs
            const bf16_t* sstg = lds + 2 * Cf::BUF + GB_STG + wid * (16 * GB_SSTG_ROW);
            bf16_t* sblk = ep.s_out + (size_t)(m0 + wm * 64 + mt * 16) * ep.ld_s + (size_t)tn * 96 + wn * 48;
            const auto rss = __builtin_amdgcn_make_buffer_rsrc(sblk, 0, 16 * ep.ld_s * 2, 0x00020000);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int e = i * 64 + lane, r = e / 6, c = e - r * 6;
              if (i == 0 || lane < 32) {
                const gb_u32x4_t v = *reinterpret_cast<const gb_u32x4_t*>(sstg + r * GB_SSTG_ROW + c * 8);
                if (flags & 2048)
                  __builtin_amdgcn_raw_buffer_store_b128(v, rss, (r * ep.ld_s + c * 8) * 2, 0, 16);
                else
                  *reinterpret_cast<gb_u32x4_t*>(sblk + (size_t)r * ep.ld_s + c * 8) = v;
              }
            }
          }
          continue;
        }
#pragma unroll
        for (int p = 0; p < NT / 2; ++p) {
          uint32_t x[2] = {pk[2 * p].x, pk[2 * p].y}, y[2] = {pk[2 * p + 1].x, pk[2 * p + 1].y};
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            auto sw = __builtin_amdgcn_permlane16_swap(x[h], y[h], false, false);
            x[h] = sw[0];
            y[h] = sw[1];
          }
          const int t = 2 * p + (lq & 1);
          const int col = gb_ncol<BN, EPI>(wn, t, ep.I) + (lq >> 1) * 8;
          const gb_u32x4_t cv = {x[0], x[1], y[0], y[1]};
          if constexpr (EPI == GB_EPI_SWIGLU_BWD) {
            // 8 consecutive ds values (bf16-rounded, as the unfused kernel reads them)
            // against the kept gate / up values of the same columns; C = dgu [M, 2I]
            gb_u32x4_t og, ou, os;
            const bool want_s = ep.s_out != nullptr;  // uniform
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              float d[2], g[2], u[2];
              gb_unpack2<HK>(cv[h], d);
              gb_unpack2<HK>(gv[mt][p][h], g);
              gb_unpack2<HK>(uv[mt][p][h], u);
              floatx4_t r, sv;
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const float sg = dlt_sigmoid(g[e]);
                r[e] = d[e] * u[e] * sg * (1.f + g[e] * (1.f - sg));
                r[2 + e] = d[e] * g[e] * sg;
                sv[e] = g[e] * sg * u[e];  // s = silu(g) * u: k_swiglu_fwd's arithmetic, same bits
                sv[2 + e] = 0.f;
              }
              const uint2 pr = gb_pack_hk<HK>(r);  // (dg0, dg1), (du0, du1)
              og[h] = pr.x;
              ou[h] = pr.y;
              os[h] = gb_pack_hk<HK>(sv).x;
            }
            // dgu has gu's layout (ldc == ld_s): the load offsets address it too
            const int so = mt * 16 * ldc * 2;
            __builtin_amdgcn_raw_buffer_store_b128(og, rs_c, sw_voff + p * 64, so, 0);
            __builtin_amdgcn_raw_buffer_store_b128(ou, rs_c, sw_voff + p * 64,
                                                   so + ep.I * 2, 0);
            // s_out (engine s ring): the down weight gradient's operand, rewritten from the
            // kept gu as k_swiglu_bwd's s_out does -- no separate k_swiglu_fwd pass
            if (want_s) *reinterpret_cast<gb_u32x4_t*>(ep.s_out + (size_t)row * ep.I + n0 + col) = os;
          } else {
            gb_u32x4_t* cp = reinterpret_cast<gb_u32x4_t*>(crow + col);
            if (flags & 128)  // nontemporal (streaming) C stores
              __builtin_nontemporal_store(cv, cp);
            else
              *cp = cv;
          }
        }
      }
      if (flags & 32) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (LATE) {
        // younger than K-tile 0's DMA: K-tile 1's A0 / B0 units (4 instructions) and the
        // epilogue's stores (ROPE: 12 per wave, STORE-form permlane or staged; SWIGLU_BWD:
        // 24, +12 with s_out) -- counted so the stores keep draining into the next tile
        // (tests/test_isa_checks.py checks these counts in the ISA)
        if constexpr (EPI == GB_EPI_ROPE) {
          asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        } else if constexpr (EPI == GB_EPI_SWIGLU_BWD) {
          if (ep.s_out != nullptr)
            asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
          else
            asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
        }
        // barrier alignment: at loop exit waves 4-7 are one barrier behind waves 0-3, so
        // waves 0-3 pass one barrier that pairs with the others' last loop barrier, then
        // all meet behind every wave's staging (the kernel prologue's state), and waves
        // 4-7 fall one barrier behind again
        if (half == 0) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_barrier();
        if (half == 1) __builtin_amdgcn_s_barrier();
      }
    }
#ifdef GB_STAMPS
    {
      const uint64_t t3 = GB_T();
      a_it0 += t1 - t0;
      a_rest += t2 - t1;
      a_epi += t3 - t2;
      ++ntl;
    }
#endif
    if (!has_next) break;
    tile = next;
  }
  // LATE: the last tile re-staged its own operands; no LDS-DMA may still be writing the
  // workgroup's LDS when it is released
  if constexpr (LATE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (half == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts for both halves
#ifdef GB_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t s_k1 = GB_T(), s_r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    unsigned long long* o = gb_stamp_buf + (size_t)(bid * 8 + wid) * 8;
    o[0] = a_it0;
    o[1] = a_rest;
    o[2] = a_epi;
    o[3] = ntl;
    o[4] = s_k1 - s_k0;
    o[5] = s_r1 - s_r0;
    o[6] = s_k0;
    o[7] = s_r0;
  }
#endif
}

// grid: one workgroup per CU (at most), a multiple of 8 (XCD-slot tile walk)
static inline int gb_grid(int ntiles) {
  int g = ntiles < 256 ? ntiles : 256;
  return (g + 7) & ~7;
}

// flags & 256: bounded persistence -- each workgroup walks at most T = max(1, (flags >> 24)
// & 15) tiles (grid = ceil(tiles / T), a multiple of 8) instead of one workgroup per CU
// for the whole launch: workgroups end every T tiles and hand their CU back to the
// dispatcher, so kernels of another stream get CUs while the GEMM runs (a persistent grid
// holds its CUs for the whole launch).  T = 1: one tile per workgroup.
// flags >> 16 (A/B knob): cap the persistent grid at 8 * (flags >> 16) workgroups, so
// kernels of the other stream keep the remaining CUs
static inline int gb_launch_grid(int ntiles, int flags) {
  if (flags & 256) {
    const int t = ((flags >> 24) & 15) ? ((flags >> 24) & 15) : 1;
    return ((ntiles + t - 1) / t + 7) & ~7;
  }
  const int g = gb_grid(ntiles), cap = 8 * ((flags >> 16) & 0xff);
  return cap && cap < g ? cap : g;
}

static inline bool gb_shape_ok(int M, int N, int K, int lda, int ldb, int ldc) {
  return M > 0 && N > 0 && M % 256 == 0 && K % 128 == 0 && K >= 128 && (lda | ldb | ldc) % 8 == 0;
}

// C = A . B^T (bf16, or IEEE half with hk = 1).  Only the 192-column tile is
// instantiated: the 256-column one needs 256 accumulator + fragment VGPRs per lane and
// spills at 8 waves per CU.
DLT_API int dlt_gemm_bf16_tn(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb,
                             int ldc, int flags, int hk, hipStream_t st) {
  if (!gb_shape_ok(M, N, K, lda, ldb, ldc) || (N % 192 && N % 128)) return -1;
  GbEpi ep{};
  if (N % 192 == 0) {
    const int ntiles = (M / 256) * (N / 192);
    DLT_HK_DISPATCH(hk, k_gemm_bf16<192, GB_EPI_STORE, false, HKC><<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(
                            A, B, C, M, N, K, lda, ldb, ldc, flags, ep));
  } else {  // 256 x 128 tiles (hidden sizes such as 1024)
    const int ntiles = (M / 256) * (N / 128);
    DLT_HK_DISPATCH(hk, k_gemm_bf16<128, GB_EPI_STORE, false, HKC><<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(
                            A, B, C, M, N, K, lda, ldb, ldc, flags, ep));
  }
  DLT_CHECK_LAUNCH();
}

// qkv[M, 3H] = x . Wqkv^T with RoPE (head_dim 64) on the q and k heads: position of
// row m = m % S, tables cos/sin [>= S, 32] fp32.
DLT_API int dlt_gemm_bf16_qkv_rope(const bf16_t* A, const bf16_t* W, bf16_t* C, int M, int H, int K, int S,
                                   const float* cosT, const float* sinT, int flags, hipStream_t st) {
  const int N = 3 * H;
  if (!gb_shape_ok(M, N, K, K, K, N) || N % 192 || H % 64 || S <= 0) return -1;
  GbEpi ep{cosT, sinT, S, 2 * H, nullptr, 0, 0};
  const int ntiles = (M / 256) * (N / 192);
  if (flags & 4096)  // epilogue-first staging of the next tile
    k_gemm_bf16<192, GB_EPI_ROPE, false, 0, true>
        <<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(A, W, C, M, N, K, K, K, N, flags, ep);
  else
    k_gemm_bf16<192, GB_EPI_ROPE><<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(A, W, C, M, N, K, K, K, N, flags, ep);
  DLT_CHECK_LAUNCH();
}

// Data gradient dX[M, Nout] = dY[M, Nred] . W[Nred, Nout] with W read as stored (the
// input gradients of every projection: q/k/v, o, gate/up, down and the tied lm_head).
// hk: operand / output format (0 bf16, 1 fp16).
DLT_API int dlt_gemm_bf16_nn(const bf16_t* dY, const bf16_t* W, bf16_t* dX, int M, int Nout, int Nred, int ldy,
                             int ldw, int ldx, int flags, int hk, hipStream_t st) {
  if (!gb_shape_ok(M, Nout, Nred, ldy, ldw, ldx) || (Nout % 192 && Nout % 128)) return -1;
  GbEpi ep{};
  if (Nout % 192 == 0) {
    const int ntiles = (M / 256) * (Nout / 192);
    DLT_HK_DISPATCH(hk, k_gemm_bf16<192, GB_EPI_STORE, true, HKC><<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(
                            dY, W, dX, M, Nout, Nred, ldy, ldw, ldx, flags, ep));
  } else {  // 256 x 128 tiles
    const int ntiles = (M / 256) * (Nout / 128);
    DLT_HK_DISPATCH(hk, k_gemm_bf16<128, GB_EPI_STORE, true, HKC><<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(
                            dY, W, dX, M, Nout, Nred, ldy, ldw, ldx, flags, ep));
  }
  DLT_CHECK_LAUNCH();
}

// Down-projection data gradient fused with the SwiGLU backward: ds = dd[M, H] . Wdown[H, I]
// (rounded to the activation format) and dgu[M, 2I] from ds and the kept gu[M, 2I]
// (k_swiglu_bwd's math).  hk: activation format (0 bf16, 1 IEEE half).
DLT_API int dlt_gemm_bf16_down_swiglu_bwd(const bf16_t* dd, const bf16_t* Wdown, const bf16_t* gu, bf16_t* dgu,
                                          bf16_t* s_out, int M, int I, int H, int flags, int hk, hipStream_t st) {
  if (!gb_shape_ok(M, I, H, H, I, 2 * I) || I % 192) return -1;
  const int ntiles = (M / 256) * (I / 192);
  GbEpi ep{nullptr, nullptr, 1, 0, s_out, 2 * I, I, gu};  // s_out (optional): s [M, I], row stride I
  if (flags & 4096) {  // epilogue-first staging of the next tile
    DLT_HK_DISPATCH(hk, k_gemm_bf16<192, GB_EPI_SWIGLU_BWD, true, HKC, true>
                            <<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(dd, Wdown, dgu, M, I, H, H, I, 2 * I,
                                                                           flags, ep));
  } else {
    DLT_HK_DISPATCH(hk, k_gemm_bf16<192, GB_EPI_SWIGLU_BWD, true, HKC>
                            <<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(dd, Wdown, dgu, M, I, H, H, I, 2 * I,
                                                                           flags, ep));
  }
  DLT_CHECK_LAUNCH();
}

// gu[M, 2I] = x . Wgu^T (gate rows [0, I), up rows [I, 2I)) and s[M, I] = silu(g) * u.
DLT_API int dlt_gemm_bf16_gu_swiglu(const bf16_t* A, const bf16_t* W, bf16_t* gu, bf16_t* s_out, int M, int I, int K,
                                    int flags, hipStream_t st) {
  const int N = 2 * I;
  if (!gb_shape_ok(M, N, K, K, K, N) || I % 96) return -1;
  GbEpi ep{nullptr, nullptr, 1, 0, s_out, I, I};
  const int ntiles = (M / 256) * (I / 96);
  k_gemm_bf16<192, GB_EPI_SWIGLU><<<gb_launch_grid(ntiles, flags), 512, 0, st>>>(A, W, gu, M, N, K, K, K, N, flags, ep);
  DLT_CHECK_LAUNCH();
}
