// Per-wave cycle stamps of the dK/dV kernel (B16 nh12 S1024, dropout 0.1): where does a
// work item's time go (prologue, diagonal tile, per full tile, epilogue) and how are the
// items dispatched over time.  Build:
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -DDLT_ATTN_TIMING \
//     tools/cpp/attn_timing.cpp -o tools/cpp/attn_timing
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
  unsigned short *q, *k, *v, *o, *dout, *dq, *dk, *dv;
  float *lse, *delta;
  unsigned* mask;
  (void)hipMalloc(&q, n * 2); (void)hipMalloc(&k, n * 2); (void)hipMalloc(&v, n * 2); (void)hipMalloc(&o, n * 2);
  (void)hipMalloc(&dout, n * 2); (void)hipMalloc(&dq, n * 2); (void)hipMalloc(&dk, n * 2); (void)hipMalloc(&dv, n * 2);
  (void)hipMalloc(&lse, (size_t)B * nh * S * 4); (void)hipMalloc(&delta, (size_t)B * nh * S * 4);
  (void)hipMalloc(&mask, (size_t)2 * B * nh * S * ((S + 31) / 32) * 4);
  fill<<<1024, 256>>>(q, n, 1); fill<<<1024, 256>>>(k, n, 2); fill<<<1024, 256>>>(v, n, 3); fill<<<1024, 256>>>(dout, n, 4);
  const int nrb = (S + 63) / 64, G = nrb * B * nh;
  unsigned long long* tim;
  (void)hipMalloc(&tim, (size_t)G * 2 * 8 * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_tim), &tim, sizeof(tim));
  const unsigned thr = 6554;
  dlt_attn_fwd(q, k, v, o, lse, mask, B, nh, S, hd, 0.125f, 77, thr, 1.f / 0.9f, 1, 0, 0);
  for (int i = 0; i < 3; ++i) dlt_attn_bwd(q, k, v, o, dout, lse, mask, delta, dq, dk, dv, B, nh, S, hd, 0.125f, 1.f / 0.9f, 0, 0);
  (void)hipMemset(tim, 0, (size_t)G * 2 * 8 * 8);
  dlt_attn_bwd(q, k, v, o, dout, lse, mask, delta, dq, dk, dv, B, nh, S, hd, 0.125f, 1.f / 0.9f, 0, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)G * 2 * 8);
  (void)hipMemcpy(h.data(), tim, h.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int g = 0; g < G; ++g)
    for (int w = 0; w < 2; ++w) {
      const unsigned long long* r = &h[((size_t)g * 2 + w) * 8];
      if (r[0]) { t0 = std::min(t0, r[0]); t1 = std::max(t1, r[4]); }
    }
  printf("dK/dV B%d S%d: %d workgroups, makespan %.0f kcyc\n", B, S, G, (t1 - t0) / 1e3);
  // by item length (tiles)
  const int maxn = nrb;
  std::vector<double> pro(maxn + 1), dia(maxn + 1), til(maxn + 1), epi(maxn + 1), start(maxn + 1), cnt(maxn + 1);
  double sum_busy = 0;
  for (int g = 0; g < G; ++g)
    for (int w = 0; w < 2; ++w) {
      const unsigned long long* r = &h[((size_t)g * 2 + w) * 8];
      if (!r[0]) continue;
      const int nt = (int)r[5];
      pro[nt] += r[1] - r[0]; dia[nt] += r[2] - r[1];
      if (nt > 1) til[nt] += (double)(r[3] - r[2]) / (nt - 1);
      epi[nt] += r[4] - r[3]; start[nt] += r[0] - t0; cnt[nt] += 1;
      sum_busy += r[4] - r[0];
    }
  printf("%6s %6s %10s %10s %12s %10s %12s\n", "tiles", "waves", "prologue", "diag", "per tile", "epilogue", "start kcyc");
  for (int nt = 1; nt <= maxn; ++nt)
    if (cnt[nt] > 0)
      printf("%6d %6.0f %10.0f %10.0f %12.0f %10.0f %12.1f\n", nt, cnt[nt], pro[nt] / cnt[nt], dia[nt] / cnt[nt],
             nt > 1 ? til[nt] / cnt[nt] : 0.0, epi[nt] / cnt[nt], start[nt] / cnt[nt] / 1e3);
  printf("wave-busy sum %.0f kcyc over %d SIMD x 2 slots -> occupancy %.2f waves/SIMD\n", sum_busy / 1e3, 1024,
         sum_busy / ((double)(t1 - t0) * 1024));
  return 0;
}
