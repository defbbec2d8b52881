// Store-path throughput of the GEMM epilogue patterns on gfx950: one 512-thread
// workgroup per CU writes a 256 x 192 bf16 tile (96 KB) per round, 16 B per lane per
// store instruction, with different lane -> address maps:
//   0: 16 rows x 64 B per instruction (4 lanes per row; gemm_bf16.hip's permlane16 form)
//   1: 8 rows x 128 B (8 lanes per row: one full cache line each)
//   2: 4 rows x 256 B
//   3: 16 rows x 32 B... as 0 but 8 B per lane (tn8's dwordx2 form)
// build: hipcc -O3 --offload-arch=gfx950 tools/cpp/store_bench.cpp -o tools/cpp/store_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int MODE>
__global__ __launch_bounds__(512) void k_store(uint16_t* C, int ldc, int rounds, int ntm) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid & 3, wn = wid >> 2;
  uint4 v = {threadIdx.x, blockIdx.x, 7u, 9u};
  for (int r = 0; r < rounds; ++r) {
    const int tile = r * gridDim.x + blockIdx.x;
    const int tm = tile % ntm, tn = tile / ntm;
    uint16_t* base = C + (size_t)(tm * 256 + wm * 64) * ldc + tn * 192 + wn * 96;
    // the wave's 64 x 96 block = 12 KB
    if (MODE == 0) {
      const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<uint4*>(base + (size_t)(mt * 16 + l16) * ldc + p * 32 + (lq & 1) * 16 + (lq >> 1) * 8) = v;
    } else if (MODE == 1) {  // 96 cols = 192 B = 1.5 lines: rows of 12 lanes
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const int e = i * 64 + lane;  // 16-B chunk index in the 64 x 12 block
        *reinterpret_cast<uint4*>(base + (size_t)(e / 12) * ldc + (e % 12) * 8) = v;
      }
    } else if (MODE == 2) {  // two waves' halves as one 384-B row: lanes 0..23 per row
      // (emulated: each wave writes whole 192 B rows, 64 lanes = 5.33 rows)
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const int e = i * 64 + lane;
        *reinterpret_cast<uint4*>(base + (size_t)(e / 12) * ldc + (e % 12) * 8) = v;
      }
    } else {
      const int l16 = lane & 15, lq = lane >> 4;
      uint2 w = {v.x, v.y};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 6; ++nt)
          *reinterpret_cast<uint2*>(base + (size_t)(mt * 16 + l16) * ldc + nt * 16 + lq * 4) = w;
    }
  }
}

int main() {
  const int ntm = 64;
  for (int ntn : {4, 16}) {
    const int M = ntm * 256, N = ntn * 192, rounds = ntm * ntn / 256;
    uint16_t* C;
    hipMalloc(&C, (size_t)M * N * 2);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 4; ++mode) {
      auto run = [&]() {
        if (mode == 0) k_store<0><<<256, 512>>>(C, N, rounds, ntm);
        if (mode == 1) k_store<1><<<256, 512>>>(C, N, rounds, ntm);
        if (mode == 2) k_store<2><<<256, 512>>>(C, N, rounds, ntm);
        if (mode == 3) k_store<3><<<256, 512>>>(C, N, rounds, ntm);
      };
      for (int i = 0; i < 3; ++i) run();
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) run();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double us = best * 1000 / 20, bytes = (double)M * N * 2;
      printf("N=%d rounds=%d mode %d: %.1f us  %.2f TB/s\n", N, rounds, mode, us, bytes / us / 1e6);
    }
    // reference: an empty launch
    hipFree(C);
  }
  return 0;
}
