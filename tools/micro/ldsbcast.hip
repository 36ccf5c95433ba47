// Throughput probe for the K^-1 matvec at full occupancy (12 waves / CU):
// D of the 15 column chunks through the DPP row_newbcast product form
// (v_fmac_f32_dpp, one 16-byte LDS chunk per lane), the other 15 - D through
// same-address ds_read_b128 broadcasts and v_pk_fma_f32, plus ~24 VALU of
// other per-iteration work.  Prints ns per wave-iteration per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../quadrupedal_loco_amd/csrc/qloco_dpp.inc"
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

template <int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
void probe(float *out, int iters) {
  __shared__ __attribute__((aligned(16))) float v[64];
  const int t = threadIdx.x;
  float k[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) k[c] = 1e-3f * (float)((t * 7 + c * 13) % 17);
  float x = 1.0f + t;
  f2v z = {0.5f, 0.25f}, y = {0.1f, 0.2f};
  for (int it = 0; it < iters; ++it) {
    v[t] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const f4v r0 = reinterpret_cast<const f4v *>(v)[t & 15];
    float a0 = 0.0f, a1 = 0.0f;
    if constexpr (D == 15) QL_DPP_MATVEC60_2(a0, a1, r0, k, 0);
    if constexpr (D == 5) QL_DPP_MATVEC20_2(a0, a1, r0, k, 0);
    if constexpr (D == 4) QL_DPP_MATVEC16_2(a0, a1, r0, k, 0);
    if constexpr (D == 3) QL_DPP_MATVEC12_2(a0, a1, r0, k, 0);
    if constexpr (D == 2) QL_DPP_MATVEC8_2(a0, a1, r0, k, 0);
    f2v a = (f2v)(0.0f), b = (f2v)(0.0f);
#pragma unroll
    for (int q = D; q < 15; ++q) {
      const f4v r = reinterpret_cast<const f4v *>(v)[q];
      a = __builtin_elementwise_fma((f2v){k[4 * q], k[4 * q + 1]}, (f2v){r.x, r.y}, a);
      b = __builtin_elementwise_fma((f2v){k[4 * q + 2], k[4 * q + 3]}, (f2v){r.z, r.w}, b);
    }
    const float acc = (a0 + a1) + ((a.x + a.y) + (b.x + b.y));
    // ~24 VALU of ADMM-style vector work
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      z = __builtin_elementwise_fma(z, (f2v)(0.9f), y * acc);
      y = __builtin_elementwise_fma(y, (f2v)(0.5f), z);
      y = (f2v){__builtin_amdgcn_fmed3f(y.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(y.y, -1.0f, 1.0f)};
    }
    x = 0.5f * x + 1e-6f * (acc + z.x + y.y);
  }
  out[blockIdx.x * 64 + t] = x;
}

template <int D>
static void run(float *d, int blocks, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0.0f;
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(probe<D>, dim3(blocks), dim3(64), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  printf("DPP chunks %2d, LDS chunks %2d: %.3f ns per wave-iteration per SIMD\n", D, 15 - D,
         ms * 1e6 / ((double)iters * blocks / 1024.0));
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int blocks = 256 * 12 * 4;
  float *d;
  if (hipMalloc(&d, sizeof(float) * blocks * 64) != hipSuccess) return 1;
  run<15>(d, blocks, iters);
  run<5>(d, blocks, iters);
  run<4>(d, blocks, iters);
  run<3>(d, blocks, iters);
  run<2>(d, blocks, iters);
  run<0>(d, blocks, iters);
  (void)hipFree(d);
  return 0;
}
