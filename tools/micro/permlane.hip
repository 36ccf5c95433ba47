// Probe of gfx950 v_permlane16_swap / v_permlane32_swap: from X = lane id,
// build S_q (q = 0..3) and print them; expected S_q[l] = 16 q + (l % 16).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(int *out) {
  const int l = threadIdx.x;
  unsigned x = l;
  auto p16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  unsigned a = p16[0], b = p16[1];
  auto pa = __builtin_amdgcn_permlane32_swap(a, a, false, false);
  auto pb = __builtin_amdgcn_permlane32_swap(b, b, false, false);
  out[6 * l + 0] = a;
  out[6 * l + 1] = b;
  out[6 * l + 2] = pa[0];
  out[6 * l + 3] = pb[0];
  out[6 * l + 4] = pa[1];
  out[6 * l + 5] = pb[1];
}
int main() {
  int *d, h[384];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 64; l += 5)
    printf("lane %2d: a %2d b %2d | pa0 %2d pb0 %2d pa1 %2d pb1 %2d\n", l, h[6 * l], h[6 * l + 1],
           h[6 * l + 2], h[6 * l + 3], h[6 * l + 4], h[6 * l + 5]);
  (void)hipFree(d);
  return 0;
}
