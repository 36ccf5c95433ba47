// Layout probe for v_mfma_f32_4x4x1_16b_f32 (CBSZ=4 broadcast of block 0's A):
// prints, per lane, D[0..3] for A_l = 1 + l, B_l = 100 * (1 + l), C = 0.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4v __attribute__((ext_vector_type(4)));
__global__ void probe(float *out, int cbsz) {
  const int l = threadIdx.x;
  const float a = 1.0f + l, b = 100.0f * (1.0f + l);
  f4v c = (f4v)(0.0f);
  if (cbsz) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 0, 0);
  else c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[4 * l + r] = c[r];
}
int main() {
  float *d, h[256];
  hipMalloc(&d, 1024);
  for (int cb = 0; cb < 2; ++cb) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, cb);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    printf("cbsz=%d\n", cb ? 4 : 0);
    for (int l = 0; l < 12; ++l) printf("lane %2d: %g %g %g %g\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
    printf("lane 63: %g %g %g %g\n", h[252], h[253], h[254], h[255]);
  }
  hipFree(d);
  return 0;
}
