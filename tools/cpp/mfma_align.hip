// Micro-benchmark: cycles per v_mfma_f32_16x16x32_bf16 in a 64-accumulator back-to-back
// stream (one wave per SIMD, 256 workgroups x 4 waves), with the A/B operand VGPRs
// 4-aligned (v[4:7], v[68:71] like hipBLASLt's loop) vs 2-mod-4 (v[6:9], v[70:73]).
// Diagnostic for csrc/gemm_fw4.hip (round 6).  build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

#define M8(A, B) \
  "v_mfma_f32_16x16x32_bf16 a[0:3], " A ", " B ", a[0:3]\n" \
  "v_mfma_f32_16x16x32_bf16 a[4:7], " A ", " B ", a[4:7]\n" \
  "v_mfma_f32_16x16x32_bf16 a[8:11], " A ", " B ", a[8:11]\n" \
  "v_mfma_f32_16x16x32_bf16 a[12:15], " A ", " B ", a[12:15]\n" \
  "v_mfma_f32_16x16x32_bf16 a[16:19], " A ", " B ", a[16:19]\n" \
  "v_mfma_f32_16x16x32_bf16 a[20:23], " A ", " B ", a[20:23]\n" \
  "v_mfma_f32_16x16x32_bf16 a[24:27], " A ", " B ", a[24:27]\n" \
  "v_mfma_f32_16x16x32_bf16 a[28:31], " A ", " B ", a[28:31]\n"

template <int V>
__global__ __launch_bounds__(256, 1) void k(unsigned long long* out, int iters) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (V == 0)
      asm volatile(M8("v[4:7]", "v[68:71]") M8("v[8:11]", "v[72:75]") M8("v[12:15]", "v[76:79]")
                       M8("v[16:19]", "v[80:83]") ::: "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                   "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v68", "v69", "v70", "v71", "v72", "v73", "v74",
                   "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "a0", "a1", "a2", "a3", "a4", "a5",
                   "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20",
                   "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31");
    else if constexpr (V == 1)
      asm volatile(M8("v[6:9]", "v[70:73]") M8("v[10:13]", "v[74:77]") M8("v[14:17]", "v[78:81]")
                       M8("v[18:21]", "v[82:85]") ::: "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                   "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v68", "v69", "v70", "v71", "v72",
                   "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "a0",
                   "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15",
                   "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29",
                   "a30", "a31");
    else  // A 2-mod-4, B 4-aligned
      asm volatile(M8("v[6:9]", "v[68:71]") M8("v[10:13]", "v[72:75]") M8("v[14:17]", "v[76:79]")
                       M8("v[18:21]", "v[80:83]") ::: "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                   "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v68", "v69", "v70", "v71", "v72",
                   "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "a0",
                   "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15",
                   "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29",
                   "a30", "a31");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 256 * 8);
  const int iters = 2000;
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (v == 0) k<0><<<256, 256>>>(d, iters);
      else if (v == 1) k<1><<<256, 256>>>(d, iters);
      else k<2><<<256, 256>>>(d, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[256];
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      double cyc = 0;
      for (int i = 0; i < 256; ++i) cyc += h[i];
      cyc /= 256.0 * iters * 32;
      printf("variant %d: %.2f cycles per MFMA, %.3f ms\n", v, cyc, ms);
    }
  }
  return 0;
}
