// Per-wave cycle accounting of the attention forward (B16 nh12 S1024, dropout 0.1): cycles
// inside the per-tile compute vs inside the per-tile DMA wait + barrier.  Build:
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -DDLT_ATTN_FWD_TIMING \
//     tools/cpp/attn_fwd_timing.cpp -o tools/cpp/attn_fwd_timing
#include "../../distributed_llm_trainer_amd/ops/csrc/attention.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
__global__ void fill(unsigned short* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = lowbias32((unsigned)i ^ seed);
    float f = ((x & 0xffffff) / 16777216.0f - 0.5f) * 4.f;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}
int main(int argc, char** argv) {
  int B = argc > 1 ? atoi(argv[1]) : 16, nh = 12, S = argc > 2 ? atoi(argv[2]) : 1024, hd = 64;
  size_t n = (size_t)B * nh * S * hd;
  unsigned short *q, *k, *v, *o;
  float* lse;
  unsigned* mask;
  (void)hipMalloc(&q, n * 2); (void)hipMalloc(&k, n * 2); (void)hipMalloc(&v, n * 2); (void)hipMalloc(&o, n * 2);
  (void)hipMalloc(&lse, (size_t)B * nh * S * 4);
  (void)hipMalloc(&mask, (size_t)2 * B * nh * S * ((S + 31) / 32) * 4);
  fill<<<1024, 256>>>(q, n, 1); fill<<<1024, 256>>>(k, n, 2); fill<<<1024, 256>>>(v, n, 3);
  const int nrb = (S + 63) / 64, G = nrb * B * nh;
  unsigned long long* tim;
  (void)hipMalloc(&tim, (size_t)G * 2 * 6 * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_ftim), &tim, sizeof(tim));
  const unsigned thr = 6554;
  for (int i = 0; i < 20; ++i) dlt_attn_fwd(q, k, v, o, lse, mask, B, nh, S, hd, 0.125f, 77, thr, 1.f / 0.9f, i == 0, 0, 0);
  (void)hipMemset(tim, 0, (size_t)G * 2 * 6 * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  dlt_attn_fwd(q, k, v, o, lse, mask, B, nh, S, hd, 0.125f, 77, thr, 1.f / 0.9f, 0, 0, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)G * 2 * 6);
  (void)hipMemcpy(h.data(), tim, h.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, t1 = 0;
  double busy = 0, comp = 0, wait = 0, tiles = 0, waves = 0;
  for (int g = 0; g < G; ++g)
    for (int w = 0; w < 2; ++w) {
      const unsigned long long* r = &h[((size_t)g * 2 + w) * 6];
      if (!r[0]) continue;
      t0 = std::min(t0, r[0]);
      t1 = std::max(t1, r[1]);
      busy += r[1] - r[0];
      comp += r[2];
      wait += r[3];
      tiles += r[4];
      waves += 1;
    }
  printf("attn fwd B%d S%d: %.1f us (event), makespan %.0f kcyc, %d workgroups, %.0f waves\n", B, S, ms * 1e3,
         (t1 - t0) / 1e3, G, waves);
  printf("per wave-tile: compute %.0f cyc, DMA wait + barrier %.0f cyc; per wave: %.1f tiles, busy %.0f cyc "
         "(outside tiles %.0f)\n", comp / tiles, wait / tiles, tiles / waves, busy / waves,
         (busy - comp - wait) / waves);
  printf("wave-busy %.0f kcyc over 1024 SIMDs -> %.2f resident waves/SIMD on average; compute %.1f %%, wait %.1f %%\n",
         busy / 1e3, busy / ((double)(t1 - t0) * 1024), 100 * comp / busy, 100 * wait / busy);
  return 0;
}
