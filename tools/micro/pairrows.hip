// Throughput probe for a two-instances-per-wave layout of the SRBD ADMM
// iteration: each 32-lane half of a wave owns one instance, each lane two
// rows of K^-1 held as fp32 pairs {K[lo][c], K[hi][c]}, the right-hand side
// written once per lane (ds_write_b64: the lane's lo / hi entries) and read
// back by same-address ds_read_b128 broadcasts (one address per half), each
// broadcast value feeding one v_pk_fma_f32 for both rows (op_sel_hi picks the
// scalar for both halves).  Against the shipped form (one instance per wave,
// one row per lane, v_fmac_f32_dpp row_newbcast fan-out).  Both carry a
// stand-in for the ~24 VALU of per-variable work per variable.  Prints ns per
// INSTANCE-iteration per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/micro/pairrows tools/micro/pairrows.hip
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

// shipped form: one instance per wave
template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
void probe_dpp(float *out, int iters) {
  extern __shared__ __attribute__((aligned(16))) float v[];  // sized to the shipped kernel's LDS (occupancy)
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
    float a0 = 0.0f, a1 = 0.0f;
    QL_DPP_MATVEC60_2(a0, a1, r0, k, 0);
    const float acc = a0 + a1;
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

// paired rows: two instances per wave, two rows per lane
template <int WPE, int NACC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
void probe_pair(float *out, int iters) {
  extern __shared__ __attribute__((aligned(16))) float vs[];  // LDS per wave sets the occupancy
  float (*v)[64] = reinterpret_cast<float (*)[64]>(vs);
  const int t = threadIdx.x, h = t >> 5, l = t & 31;
  f2v k[60];
#pragma unroll
  for (int c = 0; c < 60; ++c)
    k[c] = (f2v){1e-3f * (float)((t * 7 + c * 13) % 17), 1e-3f * (float)((t * 5 + c * 11) % 19)};
  f2v x = {1.0f + t, 2.0f + t};
  f2v z0 = {0.5f, 0.25f}, y0 = {0.1f, 0.2f}, z1 = {0.4f, 0.3f}, y1 = {0.2f, 0.1f};
  for (int it = 0; it < iters; ++it) {
    reinterpret_cast<f2v *>(v[h])[l] = x;
    wsync();
    f2v acc[NACC];
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = (f2v)(0.0f);
#pragma unroll
    for (int q = 0; q < 15; ++q) {
      const f4v r = reinterpret_cast<const f4v *>(v[h])[q];
      acc[(4 * q + 0) % NACC] = __builtin_elementwise_fma(k[4 * q + 0], (f2v)(r.x), acc[(4 * q + 0) % NACC]);
      acc[(4 * q + 1) % NACC] = __builtin_elementwise_fma(k[4 * q + 1], (f2v)(r.y), acc[(4 * q + 1) % NACC]);
      acc[(4 * q + 2) % NACC] = __builtin_elementwise_fma(k[4 * q + 2], (f2v)(r.z), acc[(4 * q + 2) % NACC]);
      acc[(4 * q + 3) % NACC] = __builtin_elementwise_fma(k[4 * q + 3], (f2v)(r.w), acc[(4 * q + 3) % NACC]);
    }
    f2v s = acc[0];
#pragma unroll
    for (int a = 1; a < NACC; ++a) s += acc[a];
    // per-variable work for both variables (packed where the two agree)
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      z0 = __builtin_elementwise_fma(z0, (f2v)(0.9f), y0 * s.x);
      z1 = __builtin_elementwise_fma(z1, (f2v)(0.9f), y1 * s.y);
      y0 = __builtin_elementwise_fma(y0, (f2v)(0.5f), z0);
      y1 = __builtin_elementwise_fma(y1, (f2v)(0.5f), z1);
      y0 = (f2v){__builtin_amdgcn_fmed3f(y0.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(y0.y, -1.0f, 1.0f)};
      y1 = (f2v){__builtin_amdgcn_fmed3f(y1.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(y1.y, -1.0f, 1.0f)};
    }
    x = 0.5f * x + 1e-6f * (s + (f2v){z0.x + y0.y, z1.x + y1.y});
  }
  out[blockIdx.x * 64 + t] = x.x + x.y;
}

// column split: one instance per wave, lane t = 32h + l owns variable t and
// holds rows l and 32 + l over the columns of its half (32h .. 32h + 31) as
// pairs; each half reads only its own variables' rhs (8 broadcasts), one
// v_permlane32_swap + add completes both rows' sums
template <int WPE, int NACC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
void probe_split(float *out, int iters) {
  extern __shared__ __attribute__((aligned(16))) float v[];
  const int t = threadIdx.x, h = t >> 5;
  f2v k[32];
#pragma unroll
  for (int c = 0; c < 32; ++c)
    k[c] = (f2v){1e-3f * (float)((t * 7 + c * 13) % 17), 1e-3f * (float)((t * 5 + c * 11) % 19)};
  float x = 1.0f + t;
  f2v z = {0.5f, 0.25f}, y = {0.1f, 0.2f};
  const f4v *vh = reinterpret_cast<const f4v *>(v) + 8 * h;
  for (int it = 0; it < iters; ++it) {
    v[t] = x;
    wsync();
    f2v acc[NACC];
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = (f2v)(0.0f);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const f4v r = vh[q];
      acc[(4 * q + 0) % NACC] = __builtin_elementwise_fma(k[4 * q + 0], (f2v)(r.x), acc[(4 * q + 0) % NACC]);
      acc[(4 * q + 1) % NACC] = __builtin_elementwise_fma(k[4 * q + 1], (f2v)(r.y), acc[(4 * q + 1) % NACC]);
      acc[(4 * q + 2) % NACC] = __builtin_elementwise_fma(k[4 * q + 2], (f2v)(r.z), acc[(4 * q + 2) % NACC]);
      acc[(4 * q + 3) % NACC] = __builtin_elementwise_fma(k[4 * q + 3], (f2v)(r.w), acc[(4 * q + 3) % NACC]);
    }
    f2v s = acc[0];
#pragma unroll
    for (int a = 1; a < NACC; ++a) s += acc[a];
    auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, s.x),
                                               __builtin_bit_cast(unsigned, s.y), false, false);
    const float acc1 = __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      z = __builtin_elementwise_fma(z, (f2v)(0.9f), y * acc1);
      y = __builtin_elementwise_fma(y, (f2v)(0.5f), z);
      y = (f2v){__builtin_amdgcn_fmed3f(y.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(y.y, -1.0f, 1.0f)};
    }
    x = 0.5f * x + 1e-6f * (acc1 + z.x + y.y);
  }
  out[blockIdx.x * 64 + t] = x;
}

template <typename F>
static double timeit(F launch, int reps = 3) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f, ms = 0.0f;
  for (int rep = 0; rep < reps; ++rep) {
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  return best;
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  float *d;
  const int maxb = 256 * 4 * 16;
  if (hipMalloc(&d, sizeof(float) * maxb * 64) != hipSuccess) return 1;
  // instances per SIMD: 4 (the headline's B = 4096) and 12 (throughput end)
  for (int ips : {1, 4, 12}) {
    const int inst = 1024 * ips;
    double ms;
    ms = timeit([&] { hipLaunchKernelGGL(probe_dpp<3>, dim3(inst), dim3(64), 13000, 0, d, iters); });
    printf("instances/SIMD %2d  dpp   3 waves/SIMD  : %.3f ns per instance-iteration per SIMD\n", ips,
           ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL(probe_dpp<2>, dim3(inst), dim3(64), 19500, 0, d, iters); });
    printf("instances/SIMD %2d  dpp   2 waves/SIMD  : %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_pair<2, 2>), dim3(inst / 2), dim3(64), 19500, 0, d, iters); });
    printf("instances/SIMD %2d  pair  2 waves/SIMD 2 acc: %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_pair<2, 4>), dim3(inst / 2), dim3(64), 19500, 0, d, iters); });
    printf("instances/SIMD %2d  pair  2 waves/SIMD 4 acc: %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_split<3, 2>), dim3(inst), dim3(64), 13000, 0, d, iters); });
    printf("instances/SIMD %2d  split 3 waves/SIMD 2 acc: %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_split<4, 2>), dim3(inst), dim3(64), 9800, 0, d, iters); });
    printf("instances/SIMD %2d  split 4 waves/SIMD 2 acc: %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_split<4, 4>), dim3(inst), dim3(64), 9800, 0, d, iters); });
    printf("instances/SIMD %2d  split 4 waves/SIMD 4 acc: %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_dpp<4>), dim3(inst), dim3(64), 9800, 0, d, iters); });
    printf("instances/SIMD %2d  dpp   4 waves/SIMD  : %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
    ms = timeit([&] { hipLaunchKernelGGL((probe_pair<1, 4>), dim3(inst / 2), dim3(64), 39000, 0, d, iters); });
    printf("instances/SIMD %2d  pair  1 wave/SIMD  4 acc: %.3f ns\n", ips, ms * 1e6 / ((double)iters * inst / 1024.0));
  }
  (void)hipFree(d);
  return 0;
}
