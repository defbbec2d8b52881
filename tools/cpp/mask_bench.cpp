// Timing of the attention keep-bit kernel (B8 nh12 S1024) -- used for layout experiments.
#include "../../distributed_llm_trainer_amd/ops/csrc/attention.hip"
#include <cstdio>
int main() {
  int B = 8, nh = 12, S = 1024, W = S / 32;
  unsigned* mask;
  hipMalloc(&mask, (size_t)2 * B * nh * S * W * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) dlt_attn_dropout_mask(mask, B, nh, S, 77, 6554, 0);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 50; ++i) dlt_attn_dropout_mask(mask, B, nh, S, 77 + i, 6554, 0);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("mask kernel %.2f us\n", ms * 1000 / 50);
  return 0;
}
