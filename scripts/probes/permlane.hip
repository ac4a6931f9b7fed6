// probe: semantics of __builtin_amdgcn_permlane32_swap on gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  const unsigned a = 100 + l, b = 200 + l;
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
}
int main() {
  unsigned* d;
  (void)hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128];
  (void)hipMemcpy(h, d, 128 * 4, hipMemcpyDeviceToHost);
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0=%u r1=%u\n", l, h[l], h[64 + l]);
  return 0;
}
