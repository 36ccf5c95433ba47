// Issue-rate probe: cycles per wave-instruction for plain v_fmac_f32,
// v_fmac_f32_dpp row_newbcast, v_pk_fma_f32 and v_fmac_f32_dpp quad_perm,
// eight independent accumulators, at 1 / 2 / 4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 dpprate.hip -o dpprate
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(X) X X X X X X X X

template <int KIND>
__global__ __launch_bounds__(64) void probe(float *out, unsigned long long *cyc, int iters) {
  const int t = threadIdx.x;
  float a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
  float b = 1.0001f + t * 1e-6f, c = 0.999f;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 0) {
      asm volatile(R8("v_fmac_f32 %0, %8, %9\n v_fmac_f32 %1, %8, %9\n v_fmac_f32 %2, %8, %9\n v_fmac_f32 %3, %8, %9\n"
                      "v_fmac_f32 %4, %8, %9\n v_fmac_f32 %5, %8, %9\n v_fmac_f32 %6, %8, %9\n v_fmac_f32 %7, %8, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b), "v"(c));
    } else if constexpr (KIND == 1) {
#define DP(i) "v_fmac_f32_dpp %" #i ", %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
      asm volatile(R8(DP(0) DP(1) DP(2) DP(3) DP(4) DP(5) DP(6) DP(7))
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b), "v"(c));
#undef DP
    } else if constexpr (KIND == 2) {
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, bb = {b, b}, cc = {c, c};
#define PK(i) "v_pk_fma_f32 %" #i ", %4, %5, %" #i "\n"
      asm volatile(R8(PK(0) PK(1) PK(2) PK(3) PK(0) PK(1) PK(2) PK(3))
                   : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)
                   : "v"(bb), "v"(cc));
#undef PK
      a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
    } else {
#define DQ(i) "v_fmac_f32_dpp %" #i ", %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      asm volatile(R8(DQ(0) DQ(1) DQ(2) DQ(3) DQ(4) DQ(5) DQ(6) DQ(7))
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b), "v"(c));
#undef DQ
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char *name, int wps) {
  const int blocks = 1024 * wps, iters = 2000;
  float *d;
  unsigned long long *c;
  (void)hipMalloc(&d, sizeof(float) * 64 * blocks);
  (void)hipMalloc(&c, sizeof(unsigned long long) * blocks);
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(64), 0, 0, d, c, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(64), 0, 0, d, c, iters);
  (void)hipEventRecord(e1);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long *h = new unsigned long long[blocks];
  (void)hipMemcpy(h, c, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  const double instr = 64.0 * iters;  // wave-instructions per wave
  printf("%-14s waves/SIMD %d: %.2f cycles/instr/wave (per-wave clock), kernel %.3f ms -> %.2f ns/instr/SIMD\n",
         name, wps, avg / instr, ms, ms * 1e6 / (instr * wps));
  delete[] h;
  (void)hipFree(d);
  (void)hipFree(c);
}

int main() {
  for (int w : {1, 2, 4}) {
    run<0>("fmac", w);
    run<1>("fmac_dpp_bc", w);
    run<2>("pk_fma", w);
    run<3>("fmac_dpp_qp", w);
  }
  return 0;
}
