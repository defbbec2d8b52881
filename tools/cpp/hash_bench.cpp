// Throughput of candidate counter-hash functions for the dropout keep bits (gfx950).
// Every thread hashes ITER consecutive counters and xor-folds the results (one store per
// thread, so the timing is pure VALU).  Prints G hashes/s per variant.
// build: hipcc -O3 --offload-arch=gfx950 tools/cpp/hash_bench.cpp -o tools/cpp/hash_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITER 256

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {  // 2 x v_mul_lo_u32
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// x * C (C < 2^24) mod 2^32 from full-rate 24-bit multiplies: x = xh * 2^24 + xl
// (inline asm: LLVM folds the split form back into one v_mul_lo_u32)
__device__ __forceinline__ uint32_t umul24(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t mul24c(uint32_t x, uint32_t c) {
  return umul24(x, c) + (umul24(x >> 24, c) << 24);  // v_mul_u32_u24 ignores bits 24-31
}
__device__ __forceinline__ uint32_t lowbias24(uint32_t x) {
  x ^= x >> 16; x = mul24c(x, 0xeb352du); x ^= x >> 15; x = mul24c(x, 0x6ca68bu); x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
// ARX mixer (add / rotate / xor only), 4 rounds of a 2-word state
__device__ __forceinline__ uint32_t arx(uint32_t k, uint32_t x) {
  uint32_t a = x, b = k;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a += b; b = rotl(b, 13) ^ a; a = rotl(a, 16);
    a += b; b = rotl(b, 17) ^ a;
  }
  return a ^ b;
}

template <int V>
__global__ void k_hash(uint32_t* out, uint32_t key) {
  const uint32_t base = (blockIdx.x * blockDim.x + threadIdx.x) * ITER;
  uint32_t acc = 0;
#pragma unroll 16
  for (int i = 0; i < ITER; ++i) {
    const uint32_t c = key ^ (base + i);
    uint32_t h;
    if (V == 0) h = lowbias32(c);
    else if (V == 1) h = lowbias24(c);
    else if (V == 2) h = arx(key, base + i);
    else h = c ^ (c >> 7) ^ (c << 9);  // no-mix floor (loop + fold overhead)
    acc ^= h + i;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int threads = 256, blocks = 256 * 64;  // 4M threads, 1G hashes per launch
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)threads * blocks * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[] = {"lowbias32 (v_mul_lo_u32)", "lowbias32 via mul_u24", "ARX 4 rounds", "no-mix floor"};
  for (int v = 0; v < 4; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0, 0);
      for (int i = 0; i < 5; ++i) {
        if (v == 0) k_hash<0><<<blocks, threads>>>(out, 77 + i);
        if (v == 1) k_hash<1><<<blocks, threads>>>(out, 77 + i);
        if (v == 2) k_hash<2><<<blocks, threads>>>(out, 77 + i);
        if (v == 3) k_hash<3><<<blocks, threads>>>(out, 77 + i);
      }
      hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("%-28s %8.1f G hashes/s (%.1f us per 1G)\n", names[v], 5.0 * threads * blocks * ITER / (ms * 1e-3) / 1e9, ms * 1000 / 5);
    }
  }
  return 0;
}
