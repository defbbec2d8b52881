// Standalone timing / correctness harness for the hand-written bf16 GEMM kernels
// (no torch import: a fresh GPU box runs it in seconds).
//   build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form \
//          -I distributed_llm_trainer_amd/ops/csrc tools/cpp/gemm_bench.cpp -lhipblaslt -o tools/cpp/gemm_bench
//   run:   tools/cpp/gemm_bench [kernel] [M N K ...]
// Operands are uniform [-1, 1) (DVFS-honest, cdna_hip_programming.md §5.4 rule 25); every
// kernel is checked against an fp32 reference on sampled rows before it is timed.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hipblaslt/hipblaslt.h>

#include "gemm_bf16.hip"
#include "elementwise.hip"
#include "gemm_wgrad.hip"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_fill(bf16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = lowbias32((uint32_t)i * 2654435761u ^ seed ^ (uint32_t)(i >> 32));
    float v = (float)(h >> 8) * (1.0f / 8388608.0f) - 1.0f;
    p[i] = f2bf(v);
  }
}

// fp32 reference of rows [r0, r0 + nr): C[m][n] = sum_k A[m][k] B[n][k]
__global__ void k_ref(const bf16_t* A, const bf16_t* B, float* C, int r0, int nr, int N, int K) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  int m = blockIdx.y;
  if (n >= N || m >= nr) return;
  const bf16_t* a = A + (size_t)(r0 + m) * K;
  const bf16_t* b = B + (size_t)n * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(a[k]) * bf2f(b[k]);
  C[(size_t)m * N + n] = s;
}

typedef int (*launch_fn)(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, hipStream_t);

template <int FLAGS>
static int run_bf16(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t s) {
  return dlt_gemm_bf16_tn(A, B, C, M, N, K, K, K, N, FLAGS, 0, s);
}

// hipBLASLt reference (system ROCm 7.2 library, best of the first 24 heuristic candidates,
// chosen once per shape): C^T[N,M] = op_T(B)[N,K] . A^T  in column-major terms
static hipblasLtHandle_t g_h = nullptr;
static void* g_ws = nullptr;
static const size_t g_wsz = 64 << 20;
struct BlasPlan {
  int M = 0, N = 0, K = 0;
  hipblasLtMatmulDesc_t md;
  hipblasLtMatrixLayout_t la, lb, lc;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
};
static BlasPlan g_plan;
static int run_blas(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t s) {
  float alpha = 1.f, beta = 0.f;
  if (!g_h) {
    hipblasLtCreate(&g_h);
    hipMalloc(&g_ws, g_wsz);
  }
  BlasPlan& p = g_plan;
  if (p.M != M || p.N != N || p.K != K) {
    p.M = M, p.N = N, p.K = K, p.ok = false;
    hipblasLtMatmulDescCreate(&p.md, HIPBLAS_COMPUTE_32F, HIP_R_32F);
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, K);
    hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, K);
    hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, N, M, N);
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &g_wsz, sizeof(g_wsz));
    hipblasLtMatmulHeuristicResult_t res[24];
    int n = 0;
    hipblasLtMatmulAlgoGetHeuristic(g_h, p.md, p.la, p.lb, p.lc, p.lc, pref, 24, res, &n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int i = 0; i < n; ++i) {
      if (res[i].workspaceSize > g_wsz) continue;
      if (hipblasLtMatmul(g_h, p.md, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo, g_ws, g_wsz, s))
        continue;
      hipEventRecord(e0, s);
      for (int j = 0; j < 5; ++j)
        hipblasLtMatmul(g_h, p.md, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo, g_ws, g_wsz, s);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms, p.algo = res[i].algo, p.ok = true;
    }
  }
  if (!p.ok) return -5;
  return (int)hipblasLtMatmul(g_h, p.md, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo, g_ws, g_wsz, s);
}

struct Kern {
  const char* name;
  launch_fn fn;
};

static float bfr(float v) {
  uint32_t u;
  memcpy(&u, &v, 4);
  u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
  memcpy(&v, &u, 4);
  return v;
}
static float bff(bf16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

template <typename F>
static float time_us(F fn, hipStream_t st, int it = 20) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) fn();
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < it; ++i) fn();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::fmin(best, ms * 1000.f / it);
  }
  return best;
}

// fused-epilogue checks (RoPE on the QKV GEMM, SwiGLU on the gate/up GEMM) against the
// fp32 reference rows + host epilogue, and timings vs hipBLASLt + the separate kernel
static int epi_main(int M, int H, int I, int S) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int K = H;
  // RoPE tables [S, 32]
  std::vector<float> hc((size_t)S * 32), hs((size_t)S * 32);
  for (int p = 0; p < S; ++p)
    for (int j = 0; j < 32; ++j) {
      float invf = 1.0f / powf(10000.f, (2.f * j) / 64.f);
      hc[p * 32 + j] = cosf(p * invf);
      hs[p * 32 + j] = sinf(p * invf);
    }
  float *dc, *ds;
  CK(hipMalloc(&dc, hc.size() * 4));
  CK(hipMalloc(&ds, hs.size() * 4));
  CK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  const int nr = 32, r0 = (M / 3) & ~7;
  for (int which = 0; which < 2; ++which) {
    const int N = which == 0 ? 3 * H : 2 * I;
    bf16_t *A, *B, *C, *C2, *Sb = nullptr, *Sb2 = nullptr;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&C2, (size_t)M * N * 2));
    if (which == 1) {
      CK(hipMalloc(&Sb, (size_t)M * I * 2));
      CK(hipMalloc(&Sb2, (size_t)M * I * 2));
    }
    k_fill<<<1024, 256, 0, st>>>(A, (size_t)M * K, 11);
    k_fill<<<1024, 256, 0, st>>>(B, (size_t)N * K, 12);
    float* R;
    CK(hipMalloc(&R, (size_t)nr * N * 4));
    k_ref<<<dim3((N + 255) / 256, nr), 256, 0, st>>>(A, B, R, r0, nr, N, K);
    std::vector<float> ref((size_t)nr * N);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    // EPI_FLAGS=n: k_gemm_bf16 flags of the fused and plain launches (1036 = LDS-transposed
    // stores + row bands, 3084 = the same with write-through stores)
    const int ef = getenv("EPI_FLAGS") ? atoi(getenv("EPI_FLAGS")) : 0;
    auto fused = [&]() {
      if (which == 0) return dlt_gemm_bf16_qkv_rope(A, B, C, M, H, K, S, dc, ds, ef, st);
      return dlt_gemm_bf16_gu_swiglu(A, B, C, Sb, M, I, K, ef, st);
    };
    auto unfused = [&]() {
      int rc = run_blas(A, B, C2, M, N, K, st);
      if (rc) return rc;
      if (which == 0) return dlt_rope_qk_inplace(C2, dc, ds, M, S, H / 64, 64, 0, st);
      return dlt_swiglu_fwd(C2, Sb2, M, I, 0, st);
    };
    CK(hipMemsetAsync(C, 0xff, (size_t)M * N * 2, st));
    if (fused() != 0) {
      printf("fused launch failed\n");
      return 1;
    }
    CK(hipStreamSynchronize(st));
    std::vector<bf16_t> got((size_t)nr * N), sgot;
    CK(hipMemcpy(got.data(), C + (size_t)r0 * N, got.size() * 2, hipMemcpyDeviceToHost));
    if (which == 1) {
      sgot.resize((size_t)nr * I);
      CK(hipMemcpy(sgot.data(), Sb + (size_t)r0 * I, sgot.size() * 2, hipMemcpyDeviceToHost));
    }
    double e1 = 0, m1 = 0, e2 = 0, m2 = 0;
    for (int r = 0; r < nr; ++r) {
      const float* rr = ref.data() + (size_t)r * N;
      const int pos = (r0 + r) % S;
      if (which == 0) {
        for (int c = 0; c < N; ++c) {
          float want = bfr(rr[c]);
          const int head = c / 64, j = c % 64;
          if (c < 2 * H) {
            const int jj = j & 31;
            const float cc = hc[pos * 32 + jj], ss = hs[pos * 32 + jj];
            const float x1 = bfr(rr[head * 64 + jj]), x2 = bfr(rr[head * 64 + jj + 32]);
            want = j < 32 ? x1 * cc - x2 * ss : x2 * cc + x1 * ss;
          }
          const double d = std::fabs((double)bff(got[(size_t)r * N + c]) - want);
          if (!(d <= e1)) e1 = d;
          m1 = std::fmax(m1, std::fabs(want));
        }
      } else {
        for (int c = 0; c < N; ++c) {
          const double d = std::fabs((double)bff(got[(size_t)r * N + c]) - rr[c]);
          if (!(d <= e1)) e1 = d;
          m1 = std::fmax(m1, std::fabs(rr[c]));
        }
        for (int c = 0; c < I; ++c) {
          const float g = bfr(rr[c]), u = bfr(rr[I + c]);
          const float want = g / (1.f + expf(-g)) * u;
          const double d = std::fabs((double)bff(sgot[(size_t)r * I + c]) - want);
          if (!(d <= e2)) e2 = d;
          m2 = std::fmax(m2, std::fabs(want));
        }
      }
    }
    const float tf = time_us(fused, st), tu = time_us(unfused, st);
    const float tp = time_us([&]() { return dlt_gemm_bf16_tn(A, B, C, M, N, K, K, K, N, ef, 0, st); }, st);
    printf("  plain bf16 %.1f us (flags %d)\n", tp, ef);
    printf("%s M=%d N=%d K=%d: fused %.1f us | hipBLASLt + %s %.1f us | err %.1e%s%.1e\n",
           which == 0 ? "qkv+rope" : "gu+swiglu", M, N, K, tf, which == 0 ? "rope" : "swiglu", tu, e1 / m1,
           which == 1 ? " s err " : "", which == 1 ? e2 / m2 : 0.0);
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(C2));
    CK(hipFree(R));
    if (Sb) CK(hipFree(Sb));
    if (Sb2) CK(hipFree(Sb2));
  }
  return 0;
}

// ---------------------------------------------------------------- data gradients
// dX[M, Nout] = dY[M, Nred] . W[Nred, Nout] (W as stored): k_gemm_bf16<.., BT = true> vs
// hipBLASLt (N, N), and the down-projection dgrad fused with the SwiGLU backward vs
// hipBLASLt + k_swiglu_bwd.
__global__ void k_ref_nn(const bf16_t* A, const bf16_t* W, float* C, int r0, int nr, int N, int K) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  int m = blockIdx.y;
  if (n >= N || m >= nr) return;
  const bf16_t* a = A + (size_t)(r0 + m) * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(a[k]) * bf2f(W[(size_t)k * N + n]);
  C[(size_t)m * N + n] = s;
}

static BlasPlan g_plan_nn;
static int run_blas_nn(const bf16_t* A, const bf16_t* W, bf16_t* C, int M, int N, int K, hipStream_t s) {
  float alpha = 1.f, beta = 0.f;
  if (!g_h) {
    hipblasLtCreate(&g_h);
    CK(hipMalloc(&g_ws, g_wsz));
  }
  BlasPlan& p = g_plan_nn;
  if (p.M != M || p.N != N || p.K != K) {
    p.M = M, p.N = N, p.K = K, p.ok = false;
    hipblasLtMatmulDescCreate(&p.md, HIPBLAS_COMPUTE_32F, HIP_R_32F);
    hipblasOperation_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, N, K, N);  // W row-major [K, N] = col-major [N, K]
    hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, K);  // dY row-major [M, K] = col-major [K, M]
    hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, N, M, N);
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &g_wsz, sizeof(g_wsz));
    hipblasLtMatmulHeuristicResult_t res[24];
    int n = 0;
    hipblasLtMatmulAlgoGetHeuristic(g_h, p.md, p.la, p.lb, p.lc, p.lc, pref, 24, res, &n);
    float best = 1e30f;
    for (int i = 0; i < n; ++i) {
      if (res[i].workspaceSize > g_wsz) continue;
      if (hipblasLtMatmul(g_h, p.md, &alpha, W, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo, g_ws, g_wsz, s))
        continue;
      const float t = time_us(
          [&]() {
            return (int)hipblasLtMatmul(g_h, p.md, &alpha, W, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo,
                                        g_ws, g_wsz, s);
          },
          s, 3);
      if (t < best) best = t, p.algo = res[i].algo, p.ok = true;
    }
  }
  if (!p.ok) return -5;
  return (int)hipblasLtMatmul(g_h, p.md, &alpha, W, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo, g_ws, g_wsz, s);
}

static int dgrad_main(std::vector<int> shp) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (size_t si = 0; si + 2 < shp.size(); si += 3) {
    const int M = shp[si], N = shp[si + 1], K = shp[si + 2];  // dX[M, N] = dY[M, K] . W[K, N]
    bf16_t *A, *W, *C;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&W, (size_t)K * N * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    k_fill<<<1024, 256, 0, st>>>(A, (size_t)M * K, 21);
    k_fill<<<1024, 256, 0, st>>>(W, (size_t)K * N, 22);
    const int nr = 32, r0 = (M / 3) & ~7;
    float* R;
    CK(hipMalloc(&R, (size_t)nr * N * 4));
    k_ref_nn<<<dim3((N + 255) / 256, nr), 256, 0, st>>>(A, W, R, r0, nr, N, K);
    std::vector<float> ref((size_t)nr * N);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const double fl = 2.0 * M * N * K;
    printf("dgrad M=%d N=%d K=%d:", M, N, K);
    for (int v = 0; v < 3; ++v) {
      auto fn = [&]() {
        if (v == 2) return run_blas_nn(A, W, C, M, N, K, st);
        return dlt_gemm_bf16_nn(A, W, C, M, N, K, K, N, N, v == 1 ? 1 : 0, 0, st);
      };
      CK(hipMemsetAsync(C, 0xff, (size_t)M * N * 2, st));
      int rc = fn();
      if (rc) {
        printf(" | v%d n/a(%d)", v, rc);
        continue;
      }
      CK(hipStreamSynchronize(st));
      double e = 0, mref = 0;
      if (v != 1) {
        std::vector<bf16_t> got((size_t)nr * N);
        CK(hipMemcpy(got.data(), C + (size_t)r0 * N, got.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < got.size(); ++i) {
          const double d = std::fabs((double)bff(got[i]) - ref[i]);
          if (!(d <= e)) e = d;
          mref = std::fmax(mref, std::fabs(ref[i]));
        }
      }
      const float t = time_us(fn, st);
      printf(" | %s %7.1f us %5.0f TF err %.1e", v == 0 ? "hand" : v == 1 ? "nostore" : "blas", t, fl / t / 1e6,
             mref > 0 ? e / mref : 0.0);
      fflush(stdout);
    }
    printf("\n");
    CK(hipFree(A));
    CK(hipFree(W));
    CK(hipFree(C));
    CK(hipFree(R));
  }
  // down dgrad + SwiGLU backward (M 16384, H 768, I 3072)
  {
    const int M = 16384, H = 768, I = 3072;
    bf16_t *dd, *Wd, *gu, *dgu, *dgu2, *ds;
    CK(hipMalloc(&dd, (size_t)M * H * 2));
    CK(hipMalloc(&Wd, (size_t)H * I * 2));
    CK(hipMalloc(&gu, (size_t)M * 2 * I * 2));
    CK(hipMalloc(&dgu, (size_t)M * 2 * I * 2));
    CK(hipMalloc(&dgu2, (size_t)M * 2 * I * 2));
    CK(hipMalloc(&ds, (size_t)M * I * 2));
    k_fill<<<1024, 256, 0, st>>>(dd, (size_t)M * H, 31);
    k_fill<<<1024, 256, 0, st>>>(Wd, (size_t)H * I, 32);
    k_fill<<<1024, 256, 0, st>>>(gu, (size_t)M * 2 * I, 33);
    const int nr = 32, r0 = (M / 3) & ~7;
    float* R;
    CK(hipMalloc(&R, (size_t)nr * I * 4));
    k_ref_nn<<<dim3((I + 255) / 256, nr), 256, 0, st>>>(dd, Wd, R, r0, nr, I, H);
    std::vector<float> ref((size_t)nr * I);
    std::vector<bf16_t> hgu((size_t)nr * 2 * I), got((size_t)nr * 2 * I);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(hgu.data(), gu + (size_t)r0 * 2 * I, hgu.size() * 2, hipMemcpyDeviceToHost, st));
    auto fused = [&]() { return dlt_gemm_bf16_down_swiglu_bwd(dd, Wd, gu, dgu, ds, M, I, H, 0, 0, st); };  // + s into ds
    auto unfused = [&]() {
      int rc = run_blas_nn(dd, Wd, ds, M, I, H, st);
      return rc ? rc : dlt_swiglu_bwd(gu, ds, dgu2, ds, M, I, 0, st);  // + s (in place over ds, as the s ring)
    };
    CK(hipMemsetAsync(dgu, 0xff, (size_t)M * 2 * I * 2, st));
    if (fused()) {
      printf("fused down+swiglu_bwd launch failed\n");
      return 1;
    }
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(got.data(), dgu + (size_t)r0 * 2 * I, got.size() * 2, hipMemcpyDeviceToHost));
    double e = 0, mref = 0;
    for (int r = 0; r < nr; ++r)
      for (int c = 0; c < I; ++c) {
        const float d = bfr(ref[(size_t)r * I + c]);
        const float g = bff(hgu[(size_t)r * 2 * I + c]), u = bff(hgu[(size_t)r * 2 * I + I + c]);
        const float sg = 1.f / (1.f + expf(-g));
        const float w0 = d * u * sg * (1.f + g * (1.f - sg)), w1 = d * g * sg;
        const double e0 = std::fabs((double)bff(got[(size_t)r * 2 * I + c]) - w0);
        const double e1 = std::fabs((double)bff(got[(size_t)r * 2 * I + I + c]) - w1);
        e = std::fmax(e, std::fmax(e0, e1));
        if (!(e0 == e0) || !(e1 == e1)) e = NAN;
        mref = std::fmax(mref, std::fmax(std::fabs(w0), std::fabs(w1)));
      }
    const float tf = time_us(fused, st), tu = time_us(unfused, st);
    const float tb = time_us([&]() { return run_blas_nn(dd, Wd, ds, M, I, H, st); }, st);
    const float th = time_us([&]() { return dlt_gemm_bf16_nn(dd, Wd, ds, M, I, H, H, I, I, 0, 0, st); }, st);
    printf("down dgrad + swiglu_bwd: fused %.1f us | hipBLASLt + k_swiglu_bwd %.1f us (dgrad alone %.1f, hand dgrad "
           "alone %.1f) | err %.1e\n",
           tf, tu, tb, th, mref > 0 ? e / mref : 0.0);
    // production flags (3084) vs epilogue-first staging (| 4096), with / without the s output;
    // each variant checked against the flags-0 result bit for bit first
    // DSW_FLAGS="f1,f2,...": the launch flags to compare (default: production 3084 and
    // epilogue-first staging 7180)
    std::vector<int> fls;
    if (const char* e = getenv("DSW_FLAGS")) {
      for (const char* c = e; *c;) {
        fls.push_back(atoi(c));
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
      }
    } else {
      fls = {3084, 3084 | 4096};
    }
    for (int fl : fls) {
      for (int ws = 0; ws < 2; ++ws) {
        auto f = [&]() { return dlt_gemm_bf16_down_swiglu_bwd(dd, Wd, gu, dgu2, ws ? ds : nullptr, M, I, H, fl, 0, st); };
        CK(hipMemsetAsync(dgu2, 0xff, (size_t)M * 2 * I * 2, st));
        if (f()) {
          printf("flags %d launch failed\n", fl);
          return 1;
        }
        CK(hipStreamSynchronize(st));
        std::vector<bf16_t> a((size_t)M * 2 * I), b((size_t)M * 2 * I);
        CK(hipMemcpy(a.data(), dgu, a.size() * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), dgu2, b.size() * 2, hipMemcpyDeviceToHost));
        const bool same = !memcmp(a.data(), b.data(), a.size() * 2);
        printf("  fused flags %d s_out %d: %.1f us  %s\n", fl, ws, time_us(f, st), same ? "bit-equal" : "MISMATCH");
        fflush(stdout);
      }
    }
  }
  return 0;
}

// dW[Nr, Nc] += dY[T, Nr]^T X[T, Nc]: hand-written wgrad (split-K partials + fixed-order
// sum) vs hipBLASLt (best of 24 heuristic candidates, fp32 C, beta = 1)
__global__ void k_ref_wgrad(const bf16_t* dY, const bf16_t* X, float* R, const int* rows, int nr, int T, int Nr,
                            int Nc) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  int ri = blockIdx.y;
  if (c >= Nc || ri >= nr) return;
  const int r = rows[ri];
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += bf2f(dY[(size_t)t * Nr + r]) * bf2f(X[(size_t)t * Nc + c]);
  R[(size_t)ri * Nc + c] = s;
}

static int wgrad_main(std::vector<int> shp) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipblasLtHandle_t h;
  hipblasLtCreate(&h);
  void* ws;
  CK(hipMalloc(&ws, g_wsz));
  for (size_t si = 0; si + 2 < shp.size(); si += 3) {
    const int T = shp[si], Nr = shp[si + 1], Nc = shp[si + 2];
    bf16_t *dY, *X;
    float *dW, *dW2, *part;
    CK(hipMalloc(&dY, (size_t)T * Nr * 2));
    CK(hipMalloc(&X, (size_t)T * Nc * 2));
    CK(hipMalloc(&dW, (size_t)Nr * Nc * 4));
    CK(hipMalloc(&dW2, (size_t)Nr * Nc * 4));
    k_fill<<<1024, 256, 0, st>>>(dY, (size_t)T * Nr, 21);
    k_fill<<<1024, 256, 0, st>>>(X, (size_t)T * Nc, 22);
    const int tiles = ((Nr + 255) / 256) * (Nc / 192);
    // GW_SPLITS=-1: the stream-K kernel (GW_GC shares per column tile, default 256 / tiles)
    int S = getenv("GW_SPLITS") ? atoi(getenv("GW_SPLITS")) : (256 + tiles / 2) / tiles;
    const int Gc = getenv("GW_GC") ? atoi(getenv("GW_GC")) : 0;
    if (S == 0) S = 1;
    const size_t nscr = S < 0 ? (size_t)dlt_gemm_wgrad_sk_scratch(T, Nr, Nc, Gc) : (size_t)S * Nr * Nc;
    CK(hipMalloc(&part, nscr * 4));
    auto hand = [&]() {
      if (S < 0) return dlt_gemm_wgrad_sk(dY, X, dW, part, T, Nr, Nc, Nr, Nc, Gc, 0, st);
      int rc = dlt_gemm_wgrad(dY, X, dW, part, T, Nr, Nc, Nr, Nc, S, 0, st);
      if (rc == 0 && S > 1) rc = dlt_splitk_acc(part, dW, (long)Nr * Nc, S, st);
      return rc;
    };
    // correctness: dW starts at 0; sampled rows vs the fp32 reference
    CK(hipMemsetAsync(dW, 0, (size_t)Nr * Nc * 4, st));
    if (hand() != 0) {
      printf("wgrad T=%d Nr=%d Nc=%d: n/a\n", T, Nr, Nc);
      continue;
    }
    const int nr = 8;
    std::vector<int> rows(nr);
    for (int i = 0; i < nr; ++i) rows[i] = (i * 977 + 13) % Nr;
    int* drows;
    float* R;
    CK(hipMalloc(&drows, nr * 4));
    CK(hipMalloc(&R, (size_t)nr * Nc * 4));
    CK(hipMemcpy(drows, rows.data(), nr * 4, hipMemcpyHostToDevice));
    k_ref_wgrad<<<dim3((Nc + 255) / 256, nr), 256, 0, st>>>(dY, X, R, drows, nr, T, Nr, Nc);
    std::vector<float> ref((size_t)nr * Nc), got((size_t)Nr * Nc);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(got.data(), dW, got.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    double maxerr = 0, maxref = 0;
    for (int i = 0; i < nr; ++i)
      for (int c = 0; c < Nc; ++c) {
        const double d = std::fabs((double)got[(size_t)rows[i] * Nc + c] - ref[(size_t)i * Nc + c]);
        if (!(d <= maxerr)) maxerr = d;
        maxref = std::fmax(maxref, std::fabs(ref[(size_t)i * Nc + c]));
      }
    if (S < 0) {  // stream-K: bitwise run-to-run, and the whole dW against the split-K kernel
      std::vector<float> again((size_t)Nr * Nc), split((size_t)Nr * Nc);
      CK(hipMemsetAsync(dW, 0, (size_t)Nr * Nc * 4, st));
      if (hand() != 0) return 1;
      CK(hipMemcpyAsync(again.data(), dW, again.size() * 4, hipMemcpyDeviceToHost, st));
      float* p2;
      CK(hipMalloc(&p2, (size_t)4 * Nr * Nc * 4));
      CK(hipMemsetAsync(dW2, 0, (size_t)Nr * Nc * 4, st));
      if (dlt_gemm_wgrad(dY, X, dW2, p2, T, Nr, Nc, Nr, Nc, 4, 0, st) || dlt_splitk_acc(p2, dW2, (long)Nr * Nc, 4, st)) return 1;
      CK(hipMemcpyAsync(split.data(), dW2, split.size() * 4, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      CK(hipFree(p2));
      double md = 0, mr = 0;
      for (size_t k = 0; k < split.size(); ++k) {
        const double d = std::fabs((double)again[k] - split[k]);
        if (!(d <= md)) md = d;
        mr = std::fmax(mr, std::fabs(split[k]));
      }
      printf("  stream-K: %s run to run, whole dW vs split-K x4 max |diff| / max %.1e, scratch %.0f MB\n",
             memcmp(again.data(), got.data(), got.size() * 4) ? "NOT bitwise" : "bitwise", md / mr, nscr * 4 / 1e6);
    }
    // hipBLASLt: C[Nc, Nr] (col-major) += op_N(X [Nc, T]) op_T(dY [Nr, T])
    hipblasLtMatmulDesc_t md;
    hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F);
    hipblasOperation_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_T;
    hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    hipblasLtMatrixLayout_t la, lb, lc;
    hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, Nc, T, Nc);
    hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, Nr, T, Nr);
    hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, Nc, Nr, Nc);
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &g_wsz, sizeof(g_wsz));
    hipblasLtMatmulHeuristicResult_t res[24];
    int n = 0;
    hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, 24, res, &n);
    float alpha = 1.f, beta = 1.f, tb_best = 1e30f;
    for (int i = 0; i < n; ++i) {
      if (res[i].workspaceSize > g_wsz) continue;
      auto blas = [&]() {
        return (int)hipblasLtMatmul(h, md, &alpha, X, la, dY, lb, &beta, dW2, lc, dW2, lc, &res[i].algo, ws, g_wsz,
                                    st);
      };
      if (blas()) continue;
      tb_best = std::fmin(tb_best, time_us(blas, st, 5));
    }
    const float th = time_us(hand, st, 5);
    const double fl = 2.0 * T * Nr * Nc;
    printf("wgrad T=%d Nr=%d Nc=%d: hand (splits %d) %7.1f us %5.0f TF err %.1e | hipBLASLt %7.1f us %5.0f TF\n", T,
           Nr, Nc, S, th, fl / th / 1e6, maxerr / maxref, tb_best, fl / tb_best / 1e6);
    fflush(stdout);
    CK(hipFree(dY));
    CK(hipFree(X));
    CK(hipFree(dW));
    CK(hipFree(dW2));
    CK(hipFree(part));
    CK(hipFree(R));
    CK(hipFree(drows));
  }
  return 0;
}

// Can memory-bound work overlap a GEMM?  hipBLASLt gate/up GEMM (G) and the SwiGLU
// elementwise kernel (E), alone, concurrently on two full-chip streams, and on
// disjoint CU masks (hipExtStreamCreateWithCUMask).
static int overlap_main() {
  const int M = 16384, N = 6144, K = 768, I = 3072;
  bf16_t *A, *B, *C, *gu, *sb;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&gu, (size_t)M * N * 2));
  CK(hipMalloc(&sb, (size_t)M * I * 2));
  k_fill<<<1024, 256>>>(A, (size_t)M * K, 1);
  k_fill<<<1024, 256>>>(B, (size_t)N * K, 2);
  k_fill<<<1024, 256>>>(gu, (size_t)M * N, 3);
  CK(hipDeviceSynchronize());
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  auto mk = [&](int lo, int hi, int stride) {  // CUs [lo, hi) (or every stride-th) -> stream
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; ++c) {
      const bool on = stride ? ((c % stride) < hi - lo) : (c >= lo && c < hi);
      if (on) m[c / 32] |= 1u << (c % 32);
    }
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    return s;
  };
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto G = [&](hipStream_t s) { return run_blas(A, B, C, M, N, K, s); };
  auto E = [&](hipStream_t s) { return dlt_swiglu_fwd(gu, sb, M, I, 0, s); };
  G(s0);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  auto wall = [&](auto&& body) {
    body();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0, 0));
      CK(hipDeviceSynchronize());
      body();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::fmin(best, ms);
    }
    return best * 1000.f / reps;
  };
  auto run = [&](const char* name, hipStream_t sg, hipStream_t se, int ne_per_g) {
    const float tg = wall([&]() { for (int i = 0; i < reps; ++i) G(sg); });
    const float te = wall([&]() { for (int i = 0; i < reps * ne_per_g; ++i) E(se); });
    const float tb = wall([&]() {
      for (int i = 0; i < reps; ++i) {
        G(sg);
        for (int j = 0; j < ne_per_g; ++j) E(se);
      }
    });
    printf("%-28s G %7.1f us | E x%d %7.1f us | both %7.1f us (serial sum %7.1f, saved %5.1f%%)\n", name, tg,
           ne_per_g, te, tb, tg + te, 100.f * (tg + te - tb) / (tg + te));
    fflush(stdout);
  };
  run("two full-chip streams", s0, s1, 1);
  run("two full-chip streams E x2", s0, s1, 2);
  for (int k : {16, 32, 64}) {
    char nm[64];
    snprintf(nm, sizeof nm, "mask G %d / E %d (low)", ncu - k, k);
    run(nm, mk(k, ncu, 0), mk(0, k, 0), 1);
    snprintf(nm, sizeof nm, "mask G %d / E %d (strided)", ncu - k, k);
    // strided: CU c in E iff c % (ncu/k) == 0
    std::vector<uint32_t> me((ncu + 31) / 32, 0u), mg((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; ++c) ((c % (ncu / k)) == 0 ? me : mg)[c / 32] |= 1u << (c % 32);
    hipStream_t sg, se;
    CK(hipExtStreamCreateWithCUMask(&sg, (uint32_t)mg.size(), mg.data()));
    CK(hipExtStreamCreateWithCUMask(&se, (uint32_t)me.size(), me.data()));
    run(nm, sg, se, 1);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "overlap")) return overlap_main();
  if (argc > 1 && !strcmp(argv[1], "epi")) return epi_main(16384, 768, 3072, 1024);
  if (argc > 1 && !strcmp(argv[1], "dgrad")) {
    std::vector<int> v;
    for (int i = 2; i < argc; ++i) v.push_back(atoi(argv[i]));
    if (v.empty()) v = {16384, 768, 2304, 16384, 768, 768, 16384, 768, 6144, 16384, 3072, 768, 16384, 768, 50304};
    return dgrad_main(v);
  }
  if (argc > 1 && !strcmp(argv[1], "wgrad")) {
    std::vector<int> v;
    for (int i = 2; i < argc; ++i) v.push_back(atoi(argv[i]));
    if (v.empty()) v = {32768, 2304, 768, 32768, 768, 768, 32768, 6144, 768, 32768, 768, 3072, 32768, 50304, 768};
    return wgrad_main(v);
  }
  std::vector<Kern> kerns = {{"blas", run_blas},         {"bf16", run_bf16<0>},      {"rowmaj", run_bf16<4>},
                             {"rowwalk", run_bf16<8>}, {"nostore", run_bf16<1>},   {"l2ops", run_bf16<2>},
                             {"l2nost", run_bf16<3>},    {"c0", run_bf16<16>},       {"stsync", run_bf16<32>},
                             {"nt", run_bf16<128>},      {"ntrow", run_bf16<132>},   {"np", run_bf16<256>},
                             {"nprow", run_bf16<260>},   {"d4", run_bf16<512 | (4 << 24)>},
                             {"d8", run_bf16<512 | (8 << 24)>}, {"d13", run_bf16<512 | (13 << 24)>},
                             {"d20", run_bf16<512 | (20 << 24)>}, {"lt", run_bf16<1024>}, {"xb", run_bf16<12>},
                             {"xblt", run_bf16<1036>}, {"sc1", run_bf16<3072>},
                             {"xbsc1", run_bf16<3084>}};
  std::string only = (argc > 1 && strcmp(argv[1], "all")) ? std::string(",") + argv[1] + "," : "all";
  std::vector<int> shp;
  for (int i = 2; i < argc; ++i) shp.push_back(atoi(argv[i]));
  if (shp.empty()) {
    int d[] = {16384, 768, 768, 16384, 768, 1536, 16384, 768, 3072, 16384, 768, 6144,
               16384, 2304, 768, 16384, 6144, 768, 16384, 3072, 768};
    shp.assign(d, d + sizeof(d) / sizeof(int));
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t si = 0; si + 2 < shp.size(); si += 3) {
    const int M = shp[si], N = shp[si + 1], K = shp[si + 2];
    bf16_t *A, *B, *C;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    k_fill<<<1024, 256, 0, st>>>(A, (size_t)M * K, 1);
    k_fill<<<1024, 256, 0, st>>>(B, (size_t)N * K, 2);
    const int nr = 64, r0 = M / 2 - 17 > 0 ? (M / 3) & ~7 : 0;
    float* R;
    CK(hipMalloc(&R, (size_t)nr * N * 4));
    k_ref<<<dim3((N + 255) / 256, nr), 256, 0, st>>>(A, B, R, r0, nr, N, K);
    std::vector<float> ref((size_t)nr * N);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const double fl = 2.0 * M * N * K;
    printf("M=%d N=%d K=%d:", M, N, K);
    for (auto& kr : kerns) {
      if (only != "all" && only.find(std::string(",") + kr.name + ",") == std::string::npos) continue;
      CK(hipMemsetAsync(C, 0xff, (size_t)M * N * 2, st));
      int rc = kr.fn(A, B, C, M, N, K, st);
      if (rc != 0) {
        printf(" | %s n/a(%d)", kr.name, rc);
        continue;
      }
      CK(hipStreamSynchronize(st));
      std::vector<bf16_t> got((size_t)nr * N);
      CK(hipMemcpy(got.data(), C + (size_t)r0 * N, got.size() * 2, hipMemcpyDeviceToHost));
      double maxerr = 0, maxref = 0;
      for (size_t i = 0; i < got.size(); ++i) {
        uint32_t u = (uint32_t)got[i] << 16;
        float g;
        memcpy(&g, &u, 4);
        double d = std::fabs((double)g - ref[i]);
        if (!(d <= maxerr)) maxerr = d;  // NaN-propagating
        maxref = std::fmax(maxref, std::fabs(ref[i]));
      }
      // full-matrix poison check on the last rows too (unwritten tiles stay 0xffff = NaN)
      std::vector<bf16_t> tail((size_t)8 * N);
      CK(hipMemcpy(tail.data(), C + (size_t)(M - 8) * N, tail.size() * 2, hipMemcpyDeviceToHost));
      int poisoned = 0;
      for (auto v : tail) poisoned += (v == 0xffff);
      for (int w = 0; w < 3; ++w) kr.fn(A, B, C, M, N, K, st);
      const int it = 20;
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < it; ++i) kr.fn(A, B, C, M, N, K, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::fmin(best, ms * 1000.f / it);
      }
      printf(" | %s %7.1f us %5.0f TF err %.1e%s", kr.name, best, fl / best / 1e6, maxerr / maxref,
             poisoned ? " POISON" : "");
      fflush(stdout);
    }
    printf("\n");
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(R));
  }
  return 0;
}
