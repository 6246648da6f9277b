// ds_permute_b32 (forward permute) semantics on gfx950: what a lane that no
// active lane writes to receives, with the writers exec-masked.
//   hipcc --offload-arch=gfx950 -O3 -o build/probe/permute scripts/debug/permute_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void probe(uint32_t* out) {
  const uint32_t l = threadIdx.x;
  uint32_t v = 0xdead0000u | l;  // the destination register's old value
  // lanes 3, 10, 40 send (100 + l) to lanes 7, 11, 63; the others are inactive
  if (l == 3 || l == 10 || l == 40) {
    const uint32_t dst = l == 3 ? 7u : (l == 10 ? 11u : 63u);
    v = __builtin_amdgcn_ds_permute(dst * 4, 100 + l);
  }
  out[l] = v;
  // all lanes active, non-senders send to themselves the value 0
  const bool s = l == 3 || l == 10 || l == 40;
  const uint32_t dst = l == 3 ? 7u : (l == 10 ? 11u : (l == 40 ? 63u : l));
  out[64 + l] = __builtin_amdgcn_ds_permute(dst * 4, s ? 100 + l : 0u);
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[128];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int k = 0; k < 2; ++k) {
    printf(k == 0 ? "masked senders:" : "all active:");
    for (int i = 0; i < 64; ++i) printf(" %d:%x", i, h[64 * k + i]);
    printf("\n");
  }
  return 0;
}
