// Probe of v_permlane32_swap / v_permlane16_swap lane semantics (gfx950):
// prints, for a few lanes, which source lanes the two results come from.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned* out) {
  const unsigned l = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(a[0], a[0], false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[1], a[1], false, false);
  out[l * 6 + 0] = a[0]; out[l * 6 + 1] = a[1];
  out[l * 6 + 2] = b[0]; out[l * 6 + 3] = b[1];
  out[l * 6 + 4] = c[0]; out[l * 6 + 5] = c[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 64 * 6 * 4);
  probe<<<1, 64>>>(d);
  unsigned h[64 * 6];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l : {0, 5, 16, 21, 32, 37, 48, 53})
    printf("lane %2d: p32 (%2u,%2u)  p16(a0) (%2u,%2u)  p16(a1) (%2u,%2u)\n", l, h[l*6], h[l*6+1], h[l*6+2], h[l*6+3], h[l*6+4], h[l*6+5]);
  return 0;
}
