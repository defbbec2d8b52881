// Exhaustive hipBLASLt sweep of every GEMM role of one GPT-2-small training step at the
// fused-chain shapes (M = 16384 rows for forward / data gradient, K = 32768 tokens for the
// deferred weight gradients): best of the first 24 heuristic candidates (what the
// planner races, ops/csrc_gemm/gemm_planner.cpp) vs best of ALL solutions returned by
// hipblaslt_ext::getAllAlgos.  Same column-major mapping as the planner (ops/gemm.py).
// Build: hipcc -O2 -std=c++17 tools/cpp/hipblaslt_allsweep.cpp -lhipblaslt -o /tmp/allsweep
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <algorithm>
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

struct Role { const char* name; int ta, tb, m, n, k, lda, ldb, ldc, cfp32; float beta; };

int main() {
  const int M = 16384, T = 32768, H = 768, I = 3072, V = 50304;
  std::vector<Role> roles = {
      {"qkv fwd", 1, 0, 3 * H, M, H, H, H, 3 * H, 0, 0.f},      {"o fwd", 1, 0, H, M, H, H, H, H, 0, 0.f},
      {"gu fwd", 1, 0, 2 * I, M, H, H, H, 2 * I, 0, 0.f},       {"down fwd", 1, 0, H, M, I, I, I, H, 0, 0.f},
      {"lm_head fwd", 1, 0, V, M, H, H, H, V, 0, 0.f},          {"qkv dgrad", 0, 0, H, M, 3 * H, H, 3 * H, H, 0, 0.f},
      {"o dgrad", 0, 0, H, M, H, H, H, H, 0, 0.f},              {"gu dgrad", 0, 0, H, M, 2 * I, H, 2 * I, H, 0, 0.f},
      {"down dgrad", 0, 0, I, M, H, I, H, I, 0, 0.f},           {"lm_head dgrad", 0, 0, H, M, V, H, V, H, 0, 0.f},
      {"gu wgrad", 0, 1, H, 2 * I, T, H, 2 * I, H, 1, 1.f},     {"down wgrad", 0, 1, I, H, T, I, H, I, 1, 1.f},
      {"lm_head wgrad", 0, 1, H, V, T, H, V, H, 1, 1.f}};
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  size_t wsz = 64 << 20; void* ws; CK(hipMalloc(&ws, wsz));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (auto& r : roles) {
    const int ar = r.ta ? r.k : r.m, ac = r.ta ? r.m : r.k, br = r.tb ? r.n : r.k, bc = r.tb ? r.k : r.n;
    void *A, *B, *C;
    CK(hipMalloc(&A, (size_t)r.lda * ac * 2)); CK(hipMalloc(&B, (size_t)r.ldb * bc * 2));
    CK(hipMalloc(&C, (size_t)r.ldc * r.n * (r.cfp32 ? 4 : 2)));
    fill_rand<<<4096, 256>>>((unsigned short*)A, (size_t)r.lda * ac, 1);
    fill_rand<<<4096, 256>>>((unsigned short*)B, (size_t)r.ldb * bc, 2);
    hipMemset(C, 0, (size_t)r.ldc * r.n * (r.cfp32 ? 4 : 2));
    hipDataType ct = r.cfp32 ? HIP_R_32F : HIP_R_16BF;
    hipblasLtMatmulDesc_t md; CK(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = r.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = r.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ar, ac, r.lda));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, br, bc, r.ldb));
    CK(hipblasLtMatrixLayoutCreate(&lc, ct, r.m, r.n, r.ldc));
    hipblasLtMatmulPreference_t pref; CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(24);
    int n = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, 24, res.data(), &n));
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF, ct, ct,
                               HIPBLAS_COMPUTE_32F, all);
    float alpha = 1.f, beta = r.beta;
    const int iters = r.name[0] == 'l' ? 3 : 8;
    auto run = [&](hipblasLtMatmulAlgo_t* algo, size_t need) -> float {
      if (need > wsz) return -1;
      for (int i = 0; i < 2; ++i)
        if (hipblasLtMatmul(h, md, &alpha, A, la, B, lb, &beta, C, lc, C, lc, algo, ws, wsz, 0) != 0) return -2;
      hipEventRecord(e0, 0);
      for (int i = 0; i < iters; ++i) hipblasLtMatmul(h, md, &alpha, A, la, B, lb, &beta, C, lc, C, lc, algo, ws, wsz, 0);
      hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); return ms * 1000.f / iters;
    };
    float best = 1e9; int bi = -1;
    for (int i = 0; i < n; ++i) { float t = run(&res[i].algo, res[i].workspaceSize); if (t > 0 && t < best) { best = t; bi = i; } }
    float bestall = 1e9; int ba = -1, valid = 0;
    for (size_t i = 0; i < all.size(); ++i) {
      size_t need = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(h, md, &alpha, la, lb, &beta, lc, lc, all[i].algo, need) != HIPBLAS_STATUS_SUCCESS) continue;
      valid++;
      float t = run(&all[i].algo, need);
      if (t > 0 && t < bestall) { bestall = t; ba = (int)i; }
    }
    double fl = 2.0 * r.m * r.n * r.k;
    printf("%-14s m=%-5d n=%-5d k=%-5d heuristic(24) best #%d %8.1f us (%5.0f TF) | all(%d/%zu) best #%d %8.1f us (%5.0f TF) | gain %.1f%%\n",
           r.name, r.m, r.n, r.k, bi, best, fl / best / 1e6, valid, all.size(), ba, bestall, fl / bestall / 1e6,
           100.0 * (best - bestall) / best);
    fflush(stdout);
    hipFree(A); hipFree(B); hipFree(C);
    hipblasLtMatmulDescDestroy(md); hipblasLtMatrixLayoutDestroy(la); hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc); hipblasLtMatmulPreferenceDestroy(pref);
  }
  return 0;
}
