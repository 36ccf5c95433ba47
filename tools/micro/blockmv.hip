// K^-1 matvec iteration probe: the shipped row-per-lane DPP form (one
// ds_read_b128 + 60 v_fmac_f32_dpp row_newbcast, half-rate) against a block
// layout (lane 16a+b holds rows 4b..4b+3 x columns 16a..16a+15, four
// same-address ds_read_b128 + 64 plain v_fmac_f32 + a permlane32/16_swap
// reduce-scatter), each with ~24 VALU of ADMM-style element work, at 1-4
// waves per SIMD.  Prints ns per wave-iteration per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 blockmv.hip -o blockmv
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../quadrupedal_loco_amd/csrc/qloco_dpp.inc"
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float elem_work(float acc, float &x, f2v &z, f2v &y) {
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    z = __builtin_elementwise_fma(z, (f2v)(0.9f), y * acc);
    y = __builtin_elementwise_fma(y, (f2v)(0.5f), z);
    y = (f2v){__builtin_amdgcn_fmed3f(y.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(y.y, -1.0f, 1.0f)};
  }
  x = 0.5f * x + 1e-6f * (acc + z.x + y.y);
  return x;
}

template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
void dpp_form(float *out, int iters) {
  __shared__ __attribute__((aligned(16))) float v[64];
  const int t = threadIdx.x;
  float k[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) k[c] = 1e-3f * (float)((t * 7 + c * 13) % 17);
  float x = 1.0f + t;
  f2v z = {0.5f, 0.25f}, y = {0.1f, 0.2f};
  for (int it = 0; it < iters; ++it) {
    v[t] = x;
    wsync();
    const f4v r0 = reinterpret_cast<const f4v *>(v)[t & 15];
    float a0, a1;
    QL_DPP_MATVEC60_2(a0, a1, r0, k, 0);
    elem_work(a0 + a1, x, z, y);
  }
  out[blockIdx.x * 64 + t] = x;
}

__device__ __forceinline__ float swap32(float &lo, float &hi) {  // lanes 32-63 of lo <-> 0-31 of hi
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, lo), __builtin_bit_cast(int, hi),
                                            false, false);
  lo = __builtin_bit_cast(float, (int)r[0]);
  hi = __builtin_bit_cast(float, (int)r[1]);
  return lo + hi;
}
__device__ __forceinline__ float swap16(float &lo, float &hi) {
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, lo), __builtin_bit_cast(int, hi),
                                            false, false);
  lo = __builtin_bit_cast(float, (int)r[0]);
  hi = __builtin_bit_cast(float, (int)r[1]);
  return lo + hi;
}

template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
void block_form(float *out, int iters) {
  __shared__ __attribute__((aligned(16))) float v[64];
  const int t = threadIdx.x;
  const int a = t >> 4, b = t & 15;
  const int m = 4 * b + a;  // matrix index of this lane's variable
  float k[4][16];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 16; ++c) k[r][c] = 1e-3f * (float)((t * 7 + (16 * r + c) * 13) % 17);
  float x = 1.0f + t;
  f2v z = {0.5f, 0.25f}, y = {0.1f, 0.2f};
  const f4v *src = reinterpret_cast<const f4v *>(v) + 4 * a;
  for (int it = 0; it < iters; ++it) {
    v[m] = x;
    wsync();
    float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
    f4v xs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xs[q] = src[q];
    // all four reads in flight together (one LDS round trip), not reg-reused
    asm volatile("" : "+v"(xs[0]), "+v"(xs[1]), "+v"(xs[2]), "+v"(xs[3]));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f4v xc = xs[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xv = e == 0 ? xc.x : (e == 1 ? xc.y : (e == 2 ? xc.z : xc.w));
        p0 = fmaf(k[0][4 * q + e], xv, p0);
        p1 = fmaf(k[1][4 * q + e], xv, p1);
        p2 = fmaf(k[2][4 * q + e], xv, p2);
        p3 = fmaf(k[3][4 * q + e], xv, p3);
      }
    }
    const float s0 = swap32(p0, p2);
    const float s1 = swap32(p1, p3);
    float s0c = s0, s1c = s1;
    const float yv = swap16(s0c, s1c);
    elem_work(yv, x, z, y);
  }
  out[blockIdx.x * 64 + t] = x;
}

template <class F>
static void run(const char *name, F kern, int wps, float *d, int iters) {
  const int blocks = 1024 * wps;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0.0f;
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  printf("%-6s waves/SIMD %d: %.3f ns per wave-iteration per SIMD (%.1f ns per iteration per wave)\n",
         name, wps, ms * 1e6 / ((double)iters * wps), ms * 1e6 / iters);
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  float *d;
  if (hipMalloc(&d, sizeof(float) * 4096 * 64) != hipSuccess) return 1;
  run("dpp", dpp_form<1>, 1, d, iters);
  run("dpp", dpp_form<2>, 2, d, iters);
  run("dpp", dpp_form<3>, 3, d, iters);
  run("dpp", dpp_form<4>, 4, d, iters);
  run("block", block_form<1>, 1, d, iters);
  run("block", block_form<2>, 2, d, iters);
  run("block", block_form<3>, 3, d, iters);
  run("block", block_form<4>, 4, d, iters);
  (void)hipFree(d);
  return 0;
}
