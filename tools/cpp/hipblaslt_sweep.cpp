// Enumerate hipBLASLt solutions for the wgrad GEMM (dW[N,K] += dY^T X, bf16 in, fp32 out,
// beta=1) and time each one.  Column-major view: C^T[K,N] = X^T[K,M] * dY[M,N]
// -> opA = N (A = X as KxM col-major, lda=K), opB = T (B = dY as NxM col-major, ldb=N).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { auto e = (x); if (e != 0) { printf("err %d at %s:%d\n", (int)e, __FILE__, __LINE__); exit(1);} } while (0)

__global__ void fill_rand(unsigned short* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = (unsigned)i * 0x9E3779B1u ^ seed; x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    float f = ((x & 0xffffff) / 16777216.0f - 0.5f) * 2.0f;   // uniform [-1, 1)
    unsigned u = __float_as_uint(f); p[i] = (unsigned short)(u >> 16);
  }
}

int main(int argc, char** argv) {
  int M = 8192;
  int shapes[][2] = {{2304, 768}, {768, 768}, {6144, 768}, {768, 3072}};
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  size_t wsz = 128 << 20; void* ws; CK(hipMalloc(&ws, wsz));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (auto& s : shapes) {
    int N = s[0], K = s[1];
    void *A, *B, *C; CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&B, (size_t)M * N * 2)); CK(hipMalloc(&C, (size_t)N * K * 4));
    fill_rand<<<2048, 256>>>((unsigned short*)A, (size_t)M * K, 1); fill_rand<<<2048, 256>>>((unsigned short*)B, (size_t)M * N, 2);
    hipMemset(C, 0, (size_t)N * K * 4);
    hipblasLtMatmulDesc_t md; CK(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_T;
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, M, K));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, N, M, N));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, K, N, K));
    hipblasLtMatmulPreference_t pref; CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(200);
    int n = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, 200, res.data(), &n));
    // all solutions via the ext API
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF, HIP_R_32F, HIP_R_32F, HIPBLAS_COMPUTE_32F, all);
    float alpha = 1.f, beta = 1.f;
    auto run = [&](hipblasLtMatmulAlgo_t* algo, size_t need) -> float {
      if (need > wsz) return -1;
      for (int i = 0; i < 3; ++i)
        if (hipblasLtMatmul(h, md, &alpha, A, la, B, lb, &beta, C, lc, C, lc, algo, ws, wsz, 0) != 0) return -2;
      hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) hipblasLtMatmul(h, md, &alpha, A, la, B, lb, &beta, C, lc, C, lc, algo, ws, wsz, 0);
      hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); return ms * 100.f;  // us per call
    };
    float t0 = run(&res[0].algo, res[0].workspaceSize);
    float best = 1e9; int bi = -1;
    for (int i = 0; i < n; ++i) { float t = run(&res[i].algo, res[i].workspaceSize); if (t > 0 && t < best) { best = t; bi = i; } }
    float bestall = 1e9; int ba = -1; int valid = 0;
    for (size_t i = 0; i < all.size(); ++i) {
      size_t need = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(h, md, &alpha, la, lb, &beta, lc, lc, all[i].algo, need) != HIPBLAS_STATUS_SUCCESS) continue;
      valid++;
      float t = run(&all[i].algo, need); if (t > 0 && t < bestall) { bestall = t; ba = (int)i; }
    }
    double fl = 2.0 * M * N * K;
    printf("wgrad N=%d K=%d: heuristic#0 %.1f us (%.0f TF) | best-of-%d heuristic %.1f us (%.0f TF) | best-of-%d/%zu all %.1f us (%.0f TF) idx %d\n",
           N, K, t0, fl / t0 / 1e6, n, best, fl / best / 1e6, valid, all.size(), bestall, fl / bestall / 1e6, ba);
    fflush(stdout);
    hipFree(A); hipFree(B); hipFree(C);
  }
  return 0;
}
