// Causal flash attention (head_dim 64) with in-kernel dropout for gfx950 MFMA.
//
// Replaces the reference's naive attention (gpt.py:230-234: Q@K^T, triu mask,
// fp32 softmax, bernoulli dropout, @V -- a [B,nh,S,S] score tensor per layer) and
// the SDPA path (gpt.py:199-206).  SURVEY §2.5 K5/K6.
//
// Design (CDNA4-first, see docs/KERNELS.md):
//  * v_mfma_f32_32x32x16_bf16 everywhere.  "Swapped" products put the softmax row
//    on the lane: S^T = K.Q^T leaves one query per lane with its keys in 16
//    accumulator registers, so row max / row sum are in-lane plus one xor-32 swap,
//    and the accumulator IS the B operand of the next product (O^T = V^T.P^T) --
//    P never touches LDS.
//  * V / dO / Q / K^T operands are read with ds_read_b64_tr_b16 (hardware transpose).
//  * K/V (fwd, dQ) and Q/dO (dK/dV) tiles are register-staged into XOR-swizzled
//    LDS, double buffered: the global loads of tile t+1 are issued before the MFMAs
//    of tile t and written to LDS after them (issue-early / write-late).
//  * Dropout masks are regenerated from a counter hash (common.h drop_bits), one
//    hash per two keys; nothing but (o, lse) is stored for backward.
//  * Backward = 3 kernels: delta = rowsum(dO*O); dK/dV (one workgroup per 128 keys,
//    dK/dV accumulated in registers); dQ (one workgroup per 128 queries,
//    recomputes S and dP) -- no fp32 atomics anywhere.
//  * Causal tile skipping; the heaviest tiles are launched first.
//
// Layouts: q, k, v, dq, dk, dv: [B*nh, S, 64] bf16;  o, do: [B, S, nh, 64] bf16
// (= the [M, H] GEMM layout);  lse, delta: [B*nh, S] fp32 (natural-log lse).
#include "common.h"

#define HD 64
#define KVB 64     // keys per staged tile (fwd / dQ)
#define QB 128     // queries per workgroup (fwd / dQ), 32 per wave
#define KB 128     // keys per workgroup (dK/dV), 32 per wave
#define QSTEP 64   // queries per staged tile (dK/dV)

typedef __attribute__((address_space(3))) shortx4_t lds_shortx4_t;

// LDS tile: [64 rows][64 bf16] = 128-B rows, 16-B chunk c of row r stored at chunk
// c ^ ((r >> 1) & 7): conflict-free ds_read_b128 row-fragment reads (see notes in
// docs/KERNELS.md), 2-way on the transposed reads.
__device__ __forceinline__ int swz_off(int row, int col) {
  return row * HD + ((((col >> 3) ^ ((row >> 1) & 7))) << 3) + (col & 7);
}

// 32x32x16 operand: 8 consecutive d of one row (row-major A or B fragment)
__device__ __forceinline__ bf16x8_t lds_row8(const bf16_t* T, int row, int col) {
  return *reinterpret_cast<const bf16x8_t*>(T + swz_off(row, col));
}

__device__ __forceinline__ shortx4_t lds_tr4(const bf16_t* T, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4_t*)(T + swz_off(row, col)));
}

// A operand of  X^T-style products:  A[d][k] with k = rows of T (keys or queries),
// permuted so that it matches accumulator registers 8s..8s+7 used as the B operand:
// element j of lane-half h <-> row 16*kk + 8*(j>>2) + 4*h + (j&3).
__device__ __forceinline__ bf16x8_t tr_frag(const bf16_t* T, int kk, int dt, int lane) {
  const int h = lane >> 5, i = lane & 15;
  const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const int r1 = 16 * kk + 4 * h + (i >> 2);
  const shortx4_t a = lds_tr4(T, r1, col);
  const shortx4_t b = lds_tr4(T, r1 + 8, col);
  typedef short shortx8_t __attribute__((ext_vector_type(8)));
  shortx8_t c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, c);
}

// accumulator registers 8s..8s+7 -> bf16 B fragment
__device__ __forceinline__ bf16x8_t acc_frag(const floatx16_t& acc, int s) {
  bf16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
  return r;
}

__device__ __forceinline__ floatx16_t mfma(const bf16x8_t& a, const bf16x8_t& b, const floatx16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// row offset (within a 32x32 tile) of accumulator register i for lane-half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Register-staged tile copy: 64 rows x 64 cols bf16 from a [*, S, 64] head (rows
// row0.., zero-filled past S), 2 chunks of 16 B per thread of a 256-thread block.
struct Stage2 { u16x8 c[2]; };
__device__ __forceinline__ void stage_load(Stage2& st, const bf16_t* __restrict__ head, int row0, int S, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u;
    const int r = c >> 3, ch = c & 7;
    if (row0 + r < S) {
      st.c[u] = *reinterpret_cast<const u16x8*>(head + (size_t)(row0 + r) * HD + ch * 8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) st.c[u].v[e] = 0;
    }
  }
}
// same, for a [B, S, nh, 64] tensor (o / do layout): row stride nh*64
__device__ __forceinline__ void stage_load_bsh(Stage2& st, const bf16_t* __restrict__ base, int row0, int S,
                                               int rstride, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u;
    const int r = c >> 3, ch = c & 7;
    if (row0 + r < S) {
      st.c[u] = *reinterpret_cast<const u16x8*>(base + (size_t)(row0 + r) * rstride + ch * 8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) st.c[u].v[e] = 0;
    }
  }
}
__device__ __forceinline__ void stage_store(const Stage2& st, bf16_t* T, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u;
    const int r = c >> 3, ch = c & 7;
    *reinterpret_cast<u16x8*>(T + swz_off(r, ch * 8)) = st.c[u];
  }
}

__device__ __forceinline__ bf16x8_t load_row8(const bf16_t* __restrict__ p, bool ok) {
  if (ok) return *reinterpret_cast<const bf16x8_t*>(p);
  bf16x8_t z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

// ============================================================================ forward
template <bool DROP>
__global__ __launch_bounds__(256) void k_attn_fwd(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                  const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                  float* __restrict__ lse, int S, int nh, float c_log2,
                                                  uint32_t key, uint32_t thr, float dscale) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * KVB * HD];  // [buf][K|V][64][64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5, ql = lane & 31;
  const int nqb = (S + QB - 1) / QB;
  const int qb = nqb - 1 - blockIdx.x;  // heaviest (last) query blocks first
  const int bh = blockIdx.y;
  const int b = bh / nh, head = bh % nh;
  const size_t hoff = (size_t)bh * S * HD;
  const int q0 = qb * QB + wid * 32;  // this wave's first query
  const int qa = q0 + ql;             // this lane's query
  const uint32_t kbh = lowbias32(key + (uint32_t)bh * 0x9E3779B9u);

  // Q^T B-operand fragments, kept in registers for the whole KV sweep
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load_row8(q + hoff + (size_t)qa * HD + 16 * s + 8 * h, qa < S);

  floatx16_t oacc[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  const int kv_end = min(S, qb * QB + QB);
  const int nkv = (kv_end + KVB - 1) / KVB;
  Stage2 sk, sv;
  stage_load(sk, k + hoff, 0, S, tid);
  stage_load(sv, v + hoff, 0, S, tid);
  stage_store(sk, lds, tid);
  stage_store(sv, lds + KVB * HD, tid);
  __syncthreads();

  for (int kb = 0; kb < nkv; ++kb) {
    const int cur = kb & 1;
    const bool more = kb + 1 < nkv;
    if (more) {
      stage_load(sk, k + hoff, (kb + 1) * KVB, S, tid);
      stage_load(sv, v + hoff, (kb + 1) * KVB, S, tid);
    }
    const bf16_t* Kt = lds + cur * 2 * KVB * HD;
    const bf16_t* Vt = Kt + KVB * HD;
    const int k0 = kb * KVB;
    if (k0 <= q0 + 31) {  // wave-uniform causal skip
      floatx16_t sacc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[t][i] = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) sacc[t] = mfma(lds_row8(Kt, 32 * t + ql, 16 * s + 8 * h), qf[s], sacc[t]);
      }
      const bool need_mask = (k0 + KVB - 1 > q0) || (k0 + KVB > S);
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float sv2 = sacc[t][i] * c_log2;
          if (need_mask) {
            const int ka = k0 + 32 * t + acc_row(i, h);
            if (ka > qa || ka >= S) sv2 = -INFINITY;
          }
          sacc[t][i] = sv2;
          mx = fmaxf(mx, sv2);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = exp2f(m_run - m_new);
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
      const uint32_t rowidx = (uint32_t)qa * (uint32_t)S;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const float p0 = exp2f(sacc[t][i] - m_new);
          const float p1 = exp2f(sacc[t][i + 1] - m_new);
          l_run += p0 + p1;
          if (DROP) {
            const uint32_t ka = (uint32_t)(k0 + 32 * t + acc_row(i, h));
            const uint32_t hsh = lowbias32(kbh ^ ((rowidx + ka) >> 1));
            sacc[t][i] = ((hsh & 0xffffu) >= thr) ? p0 * dscale : 0.f;
            sacc[t][i + 1] = ((hsh >> 16) >= thr) ? p1 * dscale : 0.f;
          } else {
            sacc[t][i] = p0;
            sacc[t][i + 1] = p1;
          }
        }
      }
      // O^T[d][q] += V^T[d][key] . P^T[key][q]
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8_t pb = acc_frag(sacc[kk >> 1], kk & 1);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) oacc[dt] = mfma(tr_frag(Vt, kk, dt, lane), pb, oacc[dt]);
      }
    }
    if (more) {
      bf16_t* Kn = lds + (cur ^ 1) * 2 * KVB * HD;
      stage_store(sk, Kn, tid);
      stage_store(sv, Kn + KVB * HD, tid);
    }
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv_l = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qa < S) {
    if (h == 0) lse[(size_t)bh * S + qa] = (m_run + log2f(l_tot)) * 0.69314718055994530942f;
    bf16_t* orow = o + (((size_t)b * S + qa) * nh + head) * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w.v[e] = f2bf(oacc[dt][4 * g + e] * inv_l);
        *reinterpret_cast<u16x4*>(orow + 32 * dt + 8 * g + 4 * h) = w;
      }
  }
}

// ============================================================================ backward
// delta[bh, q] = sum_d dO[b,q,head,d] * O[b,q,head,d]
__global__ __launch_bounds__(256) void k_attn_bwd_delta(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                                        float* __restrict__ delta, int B, int S, int nh) {
  const int rows = B * S * nh;
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const int head = r % nh;
  const int s = (r / nh) % S;
  const int b = r / (nh * S);
  const bf16_t* po = o + (size_t)r * HD;
  const bf16_t* pd = dout + (size_t)r * HD;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < HD / 8; ++c) {
    const u16x8 a = *reinterpret_cast<const u16x8*>(po + 8 * c);
    const u16x8 d = *reinterpret_cast<const u16x8*>(pd + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += bf2f(a.v[e]) * bf2f(d.v[e]);
  }
  delta[((size_t)b * nh + head) * S + s] = acc;
}

// dK, dV: one workgroup per 128 keys (32 per wave), sweep query tiles of 64.
template <bool DROP>
__global__ __launch_bounds__(256) void k_attn_bwd_dkdv(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                       const bf16_t* __restrict__ v, const bf16_t* __restrict__ dout,
                                                       const float* __restrict__ lse, const float* __restrict__ delta,
                                                       bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int S, int nh,
                                                       float c_log2, float scale, uint32_t key, uint32_t thr,
                                                       float dscale) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * QSTEP * HD];  // [buf][Q|dO][64][64]
  __shared__ __attribute__((aligned(16))) float rowc[2][2][QSTEP];          // [buf][lse2|delta][64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5, kl = lane & 31;
  const int kblk = blockIdx.x;  // early key blocks are the heaviest; they launch first
  const int bh = blockIdx.y;
  const int b = bh / nh, head = bh % nh;
  const size_t hoff = (size_t)bh * S * HD;
  const int k0 = kblk * KB + wid * 32;
  const int ka = k0 + kl;
  const uint32_t kbh = lowbias32(key + (uint32_t)bh * 0x9E3779B9u);
  const int rstride = nh * HD;
  const bf16_t* dob = dout + ((size_t)b * S * nh + head) * HD;  // row s at dob + s*rstride

  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load_row8(k + hoff + (size_t)ka * HD + 16 * s + 8 * h, ka < S);
    vf[s] = load_row8(v + hoff + (size_t)ka * HD + 16 * s + 8 * h, ka < S);
  }
  floatx16_t dka[2], dva[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) { dka[dt][i] = 0.f; dva[dt][i] = 0.f; }

  const int qt_begin = (kblk * KB) / QSTEP;
  const int nqt = (S + QSTEP - 1) / QSTEP;
  Stage2 sq, sd;
  float rl = 0.f, rd = 0.f;
  auto load_rows = [&](int t) {
    stage_load(sq, q + hoff, t * QSTEP, S, tid);
    stage_load_bsh(sd, dob, t * QSTEP, S, rstride, tid);
    if (tid < QSTEP) {
      const int qq = t * QSTEP + tid;
      rl = qq < S ? lse[(size_t)bh * S + qq] * 1.44269504088896340736f : 0.f;
      rd = qq < S ? delta[(size_t)bh * S + qq] : 0.f;
    }
  };
  auto store_rows = [&](int buf) {
    stage_store(sq, lds + buf * 2 * QSTEP * HD, tid);
    stage_store(sd, lds + buf * 2 * QSTEP * HD + QSTEP * HD, tid);
    if (tid < QSTEP) { rowc[buf][0][tid] = rl; rowc[buf][1][tid] = rd; }
  };
  if (qt_begin < nqt) {
    load_rows(qt_begin);
    store_rows(0);
  }
  __syncthreads();

  for (int t = qt_begin; t < nqt; ++t) {
    const int cur = (t - qt_begin) & 1;
    const bool more = t + 1 < nqt;
    if (more) load_rows(t + 1);
    const bf16_t* Qt = lds + cur * 2 * QSTEP * HD;
    const bf16_t* Dt = Qt + QSTEP * HD;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qs = t * QSTEP + 32 * qt;
      if (qs + 31 < k0) continue;  // fully masked (wave-uniform)
      floatx16_t sacc, pacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) { sacc[i] = 0.f; pacc[i] = 0.f; }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sacc = mfma(lds_row8(Qt, 32 * qt + kl, 16 * s + 8 * h), kf[s], sacc);
        pacc = mfma(lds_row8(Dt, 32 * qt + kl, 16 * s + 8 * h), vf[s], pacc);
      }
      // rows of the accumulators are queries qs + acc_row(i,h); lanes are keys
      const bool need_mask = (qs < k0 + 31) || (qs + 32 > S) || (k0 + 32 > S);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(&rowc[cur][0][32 * qt + 8 * g + 4 * h]);
        const float4 d4 = *reinterpret_cast<const float4*>(&rowc[cur][1][32 * qt + 8 * g + 4 * h]);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dvv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          const int qa = qs + 8 * g + 4 * h + e;
          float p = exp2f(sacc[i] * c_log2 - lv[e]);
          if (need_mask && (ka > qa || qa >= S || ka >= S)) p = 0.f;
          float dp = pacc[i];
          float pd = p;
          if (DROP) {
            const uint32_t idx = (uint32_t)qa * (uint32_t)S + (uint32_t)ka;
            const uint32_t hsh = lowbias32(kbh ^ (idx >> 1));
            const uint32_t bits = (idx & 1) ? (hsh >> 16) : (hsh & 0xffffu);
            const bool keep = bits >= thr;
            pd = keep ? p * dscale : 0.f;
            dp = keep ? dp * dscale : 0.f;
          }
          sacc[i] = pd;                   // P (dropped) for dV
          pacc[i] = p * (dp - dvv[e]);    // dS
        }
      }
      // dV^T += dO^T . Pd ;  dK^T += Q^T . dS   (sum over the 32 queries of this sub-tile)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t pb = acc_frag(sacc, s);
        const bf16x8_t sb = acc_frag(pacc, s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dva[dt] = mfma(tr_frag(Dt + 32 * qt * HD, s, dt, lane), pb, dva[dt]);
          dka[dt] = mfma(tr_frag(Qt + 32 * qt * HD, s, dt, lane), sb, dka[dt]);
        }
      }
    }
    if (more) store_rows(cur ^ 1);
    __syncthreads();
  }

  if (ka < S) {
    bf16_t* dkr = dk + hoff + (size_t)ka * HD;
    bf16_t* dvr = dv + hoff + (size_t)ka * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 wk, wv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wk.v[e] = f2bf(dka[dt][4 * g + e] * scale);
          wv.v[e] = f2bf(dva[dt][4 * g + e]);
        }
        *reinterpret_cast<u16x4*>(dkr + 32 * dt + 8 * g + 4 * h) = wk;
        *reinterpret_cast<u16x4*>(dvr + 32 * dt + 8 * g + 4 * h) = wv;
      }
  }
}

// dQ: one workgroup per 128 queries (32 per wave), sweep key tiles of 64; recomputes S, dP.
template <bool DROP>
__global__ __launch_bounds__(256) void k_attn_bwd_dq(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                     const bf16_t* __restrict__ v, const bf16_t* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     bf16_t* __restrict__ dq, int S, int nh, float c_log2, float scale,
                                                     uint32_t key, uint32_t thr, float dscale) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * KVB * HD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5, ql = lane & 31;
  const int nqb = (S + QB - 1) / QB;
  const int qb = nqb - 1 - blockIdx.x;
  const int bh = blockIdx.y;
  const int b = bh / nh, head = bh % nh;
  const size_t hoff = (size_t)bh * S * HD;
  const int q0 = qb * QB + wid * 32;
  const int qa = q0 + ql;
  const bool qok = qa < S;
  const uint32_t kbh = lowbias32(key + (uint32_t)bh * 0x9E3779B9u);

  bf16x8_t qf[4], df[4];
  const bf16_t* dorow = dout + (((size_t)b * S + (qok ? qa : 0)) * nh + head) * HD;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load_row8(q + hoff + (size_t)qa * HD + 16 * s + 8 * h, qok);
    df[s] = load_row8(dorow + 16 * s + 8 * h, qok);
  }
  const float l2 = qok ? lse[(size_t)bh * S + qa] * 1.44269504088896340736f : 0.f;
  const float dl = qok ? delta[(size_t)bh * S + qa] : 0.f;
  floatx16_t dqa[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dqa[dt][i] = 0.f;

  const int kv_end = min(S, qb * QB + QB);
  const int nkv = (kv_end + KVB - 1) / KVB;
  Stage2 sk, sv;
  stage_load(sk, k + hoff, 0, S, tid);
  stage_load(sv, v + hoff, 0, S, tid);
  stage_store(sk, lds, tid);
  stage_store(sv, lds + KVB * HD, tid);
  __syncthreads();
  const uint32_t rowidx = (uint32_t)qa * (uint32_t)S;

  for (int kb = 0; kb < nkv; ++kb) {
    const int cur = kb & 1;
    const bool more = kb + 1 < nkv;
    if (more) {
      stage_load(sk, k + hoff, (kb + 1) * KVB, S, tid);
      stage_load(sv, v + hoff, (kb + 1) * KVB, S, tid);
    }
    const bf16_t* Kt = lds + cur * 2 * KVB * HD;
    const bf16_t* Vt = Kt + KVB * HD;
    const int k0 = kb * KVB;
    if (k0 <= q0 + 31) {
      floatx16_t sacc[2], pacc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) { sacc[t][i] = 0.f; pacc[t][i] = 0.f; }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sacc[t] = mfma(lds_row8(Kt, 32 * t + ql, 16 * s + 8 * h), qf[s], sacc[t]);
          pacc[t] = mfma(lds_row8(Vt, 32 * t + ql, 16 * s + 8 * h), df[s], pacc[t]);
        }
      }
      const bool need_mask = (k0 + KVB - 1 > q0) || (k0 + KVB > S);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const int kA = k0 + 32 * t + acc_row(i, h);
          float p0 = exp2f(sacc[t][i] * c_log2 - l2);
          float p1 = exp2f(sacc[t][i + 1] * c_log2 - l2);
          if (need_mask) {
            if (kA > qa || kA >= S) p0 = 0.f;
            if (kA + 1 > qa || kA + 1 >= S) p1 = 0.f;
          }
          float dp0 = pacc[t][i], dp1 = pacc[t][i + 1];
          if (DROP) {
            const uint32_t hsh = lowbias32(kbh ^ ((rowidx + (uint32_t)kA) >> 1));
            dp0 = ((hsh & 0xffffu) >= thr) ? dp0 * dscale : 0.f;
            dp1 = ((hsh >> 16) >= thr) ? dp1 * dscale : 0.f;
          }
          pacc[t][i] = p0 * (dp0 - dl);
          pacc[t][i + 1] = p1 * (dp1 - dl);
        }
      }
      // dQ^T[d][q] += K^T[d][key] . dS^T[key][q]
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8_t sb = acc_frag(pacc[kk >> 1], kk & 1);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) dqa[dt] = mfma(tr_frag(Kt, kk, dt, lane), sb, dqa[dt]);
      }
    }
    if (more) {
      bf16_t* Kn = lds + (cur ^ 1) * 2 * KVB * HD;
      stage_store(sk, Kn, tid);
      stage_store(sv, Kn + KVB * HD, tid);
    }
    __syncthreads();
  }
  if (qok) {
    bf16_t* dqr = dq + hoff + (size_t)qa * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w.v[e] = f2bf(dqa[dt][4 * g + e] * scale);
        *reinterpret_cast<u16x4*>(dqr + 32 * dt + 8 * g + 4 * h) = w;
      }
  }
}

// ============================================================================ launchers
DLT_API int dlt_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int nh,
                         int S, int hd, float scale, uint32_t key, uint32_t thr, float dscale, hipStream_t st) {
  if (hd != HD || S <= 0) return -1;
  const dim3 grid((S + QB - 1) / QB, B * nh);
  const float c_log2 = scale * 1.44269504088896340736f;
  if (thr)
    k_attn_fwd<true><<<grid, 256, 0, st>>>(q, k, v, o, lse, S, nh, c_log2, key, thr, dscale);
  else
    k_attn_fwd<false><<<grid, 256, 0, st>>>(q, k, v, o, lse, S, nh, c_log2, key, thr, dscale);
  DLT_CHECK_LAUNCH();
}

DLT_API int dlt_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                         const float* lse, float* delta_ws, bf16_t* dq, bf16_t* dk, bf16_t* dv, int B, int nh, int S,
                         int hd, float scale, uint32_t key, uint32_t thr, float dscale, hipStream_t st) {
  if (hd != HD || S <= 0) return -1;
  const int rows = B * S * nh;
  k_attn_bwd_delta<<<(rows + 255) / 256, 256, 0, st>>>(o, dout, delta_ws, B, S, nh);
  const float c_log2 = scale * 1.44269504088896340736f;
  const dim3 gk((S + KB - 1) / KB, B * nh);
  const dim3 gq((S + QB - 1) / QB, B * nh);
  if (thr) {
    k_attn_bwd_dkdv<true><<<gk, 256, 0, st>>>(q, k, v, dout, lse, delta_ws, dk, dv, S, nh, c_log2, scale, key, thr, dscale);
    k_attn_bwd_dq<true><<<gq, 256, 0, st>>>(q, k, v, dout, lse, delta_ws, dq, S, nh, c_log2, scale, key, thr, dscale);
  } else {
    k_attn_bwd_dkdv<false><<<gk, 256, 0, st>>>(q, k, v, dout, lse, delta_ws, dk, dv, S, nh, c_log2, scale, key, thr, dscale);
    k_attn_bwd_dq<false><<<gq, 256, 0, st>>>(q, k, v, dout, lse, delta_ws, dq, S, nh, c_log2, scale, key, thr, dscale);
  }
  DLT_CHECK_LAUNCH();
}
