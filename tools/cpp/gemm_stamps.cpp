// Where a persistent k_gemm_bf16 tile spends its cycles (diagnostic build, GB_STAMPS):
// per wave, s_memtime sums of the first K-iteration of each tile (8 phases, the one whose
// phase-4 vmcnt wait sits behind the previous tile's C stores), the remaining K-iterations,
// and the epilogue; plus the in-kernel clock (s_memtime / s_memrealtime x 100 MHz).
//   build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form \
//          -I distributed_llm_trainer_amd/ops/csrc tools/cpp/gemm_stamps.cpp -o tools/cpp/gemm_stamps
//   run:   tools/cpp/gemm_stamps M N K flags [flags ...]
// Operands uniform [-1, 1) (DVFS-honest); ~1.5 s of back-to-back launches before the
// measured one (cdna_hip_programming.md §7 / MI355X_MICROARCH.md 'DVFS give-back' item 6).
#define GB_STAMPS 1
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gemm_bf16.hip"

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

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s M N K flags...\n", argv[0]);
    return 2;
  }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  bf16_t *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  k_fill<<<1024, 256, 0, st>>>(A, (size_t)M * K, 1);
  k_fill<<<1024, 256, 0, st>>>(B, (size_t)N * K, 2);
  // EPI=rope (N = 3H, RoPE epilogue, S = 1024) | swiglu (N = 2I, SwiGLU epilogue) | plain
  const char* epi = getenv("EPI") ? getenv("EPI") : "plain";
  const int mode = !strcmp(epi, "rope") ? 1 : !strcmp(epi, "swiglu") ? 2 : 0;
  float* tab = nullptr;
  bf16_t* Sb = nullptr;
  if (mode == 1) {
    CK(hipMalloc(&tab, 1024 * 32 * 4));
    CK(hipMemset(tab, 0, 1024 * 32 * 4));
  }
  if (mode == 2) CK(hipMalloc(&Sb, (size_t)M * (N / 2) * 2));
  const int ntiles = (M / 256) * (mode == 2 ? N / 192 : N / 192);
  const int G = gb_grid(ntiles);
  unsigned long long* buf;
  CK(hipMalloc(&buf, (size_t)G * 8 * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(gb_stamp_buf), &buf, sizeof(buf)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("M=%d N=%d K=%d tiles=%d grid=%d epilogue %s\n", M, N, K, ntiles, G, epi);
  for (int a = 4; a < argc; ++a) {
    const int flags = atoi(argv[a]);
    // warm: ~1.5 s of launches
    float ms = 0;
    int iters = 0;
    CK(hipEventRecord(e0, st));
    while (ms < 1500.f) {
      for (int i = 0; i < 50; ++i) {
        if (mode == 1)
          dlt_gemm_bf16_qkv_rope(A, B, C, M, N / 3, K, 1024, tab, tab, flags, st);
        else if (mode == 2)
          dlt_gemm_bf16_gu_swiglu(A, B, C, Sb, M, N / 2, K, flags, st);
        else
          dlt_gemm_bf16_tn(A, B, C, M, N, K, K, K, N, flags, 0, st);
      }
      iters += 50;
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    const float us = ms * 1000.f / iters;
    std::vector<unsigned long long> h((size_t)G * 64);
    CK(hipMemcpy(h.data(), buf, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> it0, rest, epi, clk, span;
    const int nk2 = K / 128;
    for (int w = 0; w < G * 8; ++w) {
      const unsigned long long* o = &h[(size_t)w * 8];
      if (!o[3]) continue;
      it0.push_back((double)o[0] / o[3]);
      rest.push_back(nk2 > 1 ? (double)o[1] / o[3] / (nk2 - 1) : 0.0);
      epi.push_back((double)o[2] / o[3]);
      clk.push_back(o[5] ? (double)o[4] / o[5] * 100.0 : 0.0);
      span.push_back((double)o[4]);
    }
    const double i0 = med(it0), r = med(rest), e = med(epi);
    printf("flags=%d: %.1f us/launch (avg of %d) | per tile: first K-iter %.0f cyc, later K-iter %.0f cyc, "
           "epilogue %.0f cyc; first-iter excess %.0f cyc; tile = %.0f cyc | clock %.0f MHz | wave span %.0f cyc\n",
           flags, us, iters, i0, r, e, i0 - r, i0 + r * (nk2 - 1) + e, med(clk), med(span));
    fflush(stdout);
  }
  return 0;
}
