// Weight-gradient GEMMs (dW[N,K] += dY^T X, bf16 in, fp32 C accumulated, beta = 1) at
// the deferred length M = GA*B*S = 32768: heuristic candidates x user split-K
// (hipblaslt_ext::GemmTuning) -- does a split-K variant beat the plain solutions on
// the small-output shapes?  Column-major view: C^T[K,N] = X^T[K,M] * dY[M,N].
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { auto e = (x); if (e != 0) { printf("err %d at %s:%d\n", (int)e, __FILE__, __LINE__); exit(1);} } while (0)

__global__ void fill_rand(unsigned short* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = (unsigned)i * 0x9E3779B1u ^ seed; x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    float f = ((x & 0xffffff) / 16777216.0f - 0.5f) * 2.0f;
    unsigned u = __float_as_uint(f); p[i] = (unsigned short)(u >> 16);
  }
}

int main() {
  const int M = 32768;
  int shapes[][2] = {{768, 768}, {2304, 768}, {768, 3072}, {6144, 768}};  // (N, K) of dW[N,K]
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  size_t wsz = 128 << 20; void* ws; CK(hipMalloc(&ws, wsz));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipStream_t st; hipStreamCreate(&st);
  for (auto& s : shapes) {
    int N = s[0], K = s[1];
    void *A, *B, *C; CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&B, (size_t)M * N * 2)); CK(hipMalloc(&C, (size_t)N * K * 4));
    fill_rand<<<2048, 256>>>((unsigned short*)A, (size_t)M * K, 1); fill_rand<<<2048, 256>>>((unsigned short*)B, (size_t)M * N, 2);
    hipMemset(C, 0, (size_t)N * K * 4); hipDeviceSynchronize();
    hipblasLtMatmulDesc_t md; CK(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_T;
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, M, K));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, N, M, N));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, K, N, K));
    float alpha = 1.f, beta = 1.f;
    hipblaslt_ext::Gemm gemm(h, md, &alpha, A, la, B, lb, &beta, C, lc, C, lc);
    hipblaslt_ext::GemmPreference pref; pref.setMaxWorkspaceBytes(wsz);
    std::vector<hipblasLtMatmulHeuristicResult_t> res;
    CK(gemm.algoGetHeuristic(64, pref, res));
    double fl = 2.0 * M * N * K;
    float best0 = 1e9, best = 1e9; int bi = -1, bs = -1;
    for (size_t i = 0; i < res.size(); ++i) {
      for (int sk : {0, 2, 3, 4, 6, 8, 12, 16}) {
        hipblaslt_ext::GemmTuning tun; tun.setSplitK(sk);
        size_t need = 0;
        if (gemm.isAlgoSupported(res[i].algo, tun, need) != HIPBLAS_STATUS_SUCCESS || need > wsz) continue;
        if (gemm.initialize(res[i].algo, tun, ws, false, st) != HIPBLAS_STATUS_SUCCESS) continue;
        for (int w = 0; w < 2; ++w) gemm.run(st);
        hipEventRecord(e0, st);
        for (int it = 0; it < 10; ++it) gemm.run(st);
        hipEventRecord(e1, st); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        float us = ms * 100.f;
        if (sk == 0 && us < best0) best0 = us;
        if (us < best) { best = us; bi = (int)i; bs = sk; }
      }
    }
    printf("wgrad N=%d K=%d M=%d: %zu heuristic algos | best plain %.1f us (%.0f TF) | best w/ splitK %.1f us (%.0f TF) algo %d splitK %d\n",
           N, K, M, res.size(), best0, fl / best0 / 1e6, best, fl / best / 1e6, bi, bs);
    fflush(stdout);
    hipFree(A); hipFree(B); hipFree(C);
  }
  return 0;
}
