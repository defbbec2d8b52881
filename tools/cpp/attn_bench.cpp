// Standalone timing of the attention forward kernel at B8 nh12 S1024 hd64 (random data).
#include "../../distributed_llm_trainer_amd/ops/csrc/attention.hip"
#include <cstdio>
#include <vector>
__global__ void fill(unsigned short* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = lowbias32((unsigned)i ^ seed);
    float f = ((x & 0xffffff) / 16777216.0f - 0.5f) * 4.f;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}
int main() {
  int B = 8, nh = 12, S = 1024, hd = 64;
  size_t n = (size_t)B * nh * S * hd;
  unsigned short *q, *k, *v, *o; float* lse; unsigned* mask;
  hipMalloc(&q, n * 2); hipMalloc(&k, n * 2); hipMalloc(&v, n * 2); hipMalloc(&o, n * 2);
  hipMalloc(&lse, (size_t)B * nh * S * 4); hipMalloc(&mask, (size_t)2 * B * nh * S * (S / 32) * 4);
  fill<<<1024, 256>>>(q, n, 1); fill<<<1024, 256>>>(k, n, 2); fill<<<1024, 256>>>(v, n, 3);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int drop = 0; drop < 2; ++drop) {
    unsigned thr = drop ? 6554 : 0;
    for (int i = 0; i < 3; ++i) dlt_attn_fwd(q, k, v, o, lse, mask, B, nh, S, hd, 0.125f, 77, thr, 1.f / 0.9f, 1, 0, 0);
    hipEventRecord(e0, 0);
    for (int i = 0; i < 20; ++i) dlt_attn_fwd(q, k, v, o, lse, mask, B, nh, S, hd, 0.125f, 77, thr, 1.f / 0.9f, 1, 0, 0);
    hipEventRecord(e1, 0); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("dropout=%d fwd %.1f us\n", drop, ms * 1000 / 20);
  }
  return 0;
}
