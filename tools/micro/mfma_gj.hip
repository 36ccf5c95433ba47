// MFMA blocked Gauss-Jordan inverse vs the register-row DPP Gauss-Jordan of
// srbd_admm_kernel<1> (the KKT inverse of the SRBD ADMM, n <= 60 + identity
// padding to 64).  One 64x64 SPD matrix per wavefront, row layout in and out
// (lane v holds row v), as the ADMM matvec wants it.
//
// MFMA form: the matrix is held as 4x4 blocks of 16x16 in the C/D layout of
// v_mfma_f32_16x16x4_f32 (lane (j, g) = 16g + j, register r holds
// M[16I + 4g + r][16J + j]).  Block Gauss-Jordan, no pivoting (SPD):
//   P = M_kk^-1 (16-pivot GJ inside the C layout: pivot row by ds_bpermute,
//   pivot column by DPP row_newbcast),  T_J = P M_kJ,  M_IJ -= M_Ik T_J,
//   M_Ik = -M_Ik P,  M_kJ = T_J,  M_kk = P.
// The A operand of 16x16x4 wants the TRANSPOSE of a C-layout block; GJ on a
// symmetric matrix keeps M_Ik = s M_kI^T (s = -1 iff exactly one of I, k is
// processed), so the old row block k serves as every A operand.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../quadrupedal_loco_amd/csrc mfma_gj.hip -o mfma_gj
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "qloco_dpp.inc"

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------- the product DPP Gauss-Jordan (invert_w1<true>)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void gj_dpp(const float *in, float *out, int reps) {
  __shared__ __attribute__((aligned(16))) f4v bc[2][16];
  const int t = threadIdx.x, lane = t;
  const int64_t b = blockIdx.x;
  float K[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) K[c] = in[(b & 255) * 4096 + t * 64 + c];
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      const int buf = k & 1;
      float *bcf = reinterpret_cast<float *>(&bc[buf][0]);
      int tt = t;
      asm volatile("" : "+v"(tt));
      const float v = K[k];
      const float p = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
      float e = (tt < k) ? -v : v;
      e = (tt == k) ? p + 1.0f : e;
      bcf[tt] = e;
      wsync();
      const f4v r0 = bc[buf][lane & 15];
      const float pinv = __builtin_amdgcn_rcpf(p);
      const float g = (tt == k) ? (1.0f - pinv) : v * pinv;
      const float ng = -g;
      QL_DPP_GJ60(K, 0, r0, ng);
    }
    wsync();
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) out[b * 4096 + t * 64 + c] = K[c];
}

// ---------------- MFMA blocked form
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// 16-pivot GJ of one C-layout 16x16 block (in place -> its inverse)
template <int P>
__device__ __forceinline__ void diag_pivot(f4v &B, int lane) {
  constexpr int gq = P >> 2, rq = P & 3;
  const float prow = B[rq];  // M[4g + rq][j]
  const float piv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, prow), 16 * gq + P));
  const float pinv = __builtin_amdgcn_rcpf(piv);
  // pivot row entry j of this lane: lane (j, gq), register rq
  float e = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * (16 * gq + (lane & 15)), __builtin_bit_cast(int, prow)));
  e = ((lane & 15) == P) ? piv + 1.0f : e;
  const bool prow_grp = (lane >> 4) == gq;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float c = dppf<0x150 + P>(B[r]);  // M[4g + r][P]: lane P of this 16-lane row
    float g = c * pinv;
    if (r == rq) g = prow_grp ? (1.0f - pinv) : g;
    B[r] = fmaf(-g, e, B[r]);
  }
}
__device__ __forceinline__ void diag_inverse(f4v &B, int lane) {
  diag_pivot<0>(B, lane); diag_pivot<1>(B, lane); diag_pivot<2>(B, lane); diag_pivot<3>(B, lane);
  diag_pivot<4>(B, lane); diag_pivot<5>(B, lane); diag_pivot<6>(B, lane); diag_pivot<7>(B, lane);
  diag_pivot<8>(B, lane); diag_pivot<9>(B, lane); diag_pivot<10>(B, lane); diag_pivot<11>(B, lane);
  diag_pivot<12>(B, lane); diag_pivot<13>(B, lane); diag_pivot<14>(B, lane); diag_pivot<15>(B, lane);
}

// D = Z^T Y + C for C-layout blocks Z (A operand) and Y (B operand)
__device__ __forceinline__ f4v mm(const f4v &Z, const f4v &Y, f4v C) {
  C = __builtin_amdgcn_mfma_f32_16x16x4f32(Z[0], Y[0], C, 0, 0, 0);
  C = __builtin_amdgcn_mfma_f32_16x16x4f32(Z[1], Y[1], C, 0, 0, 0);
  C = __builtin_amdgcn_mfma_f32_16x16x4f32(Z[2], Y[2], C, 0, 0, 0);
  C = __builtin_amdgcn_mfma_f32_16x16x4f32(Z[3], Y[3], C, 0, 0, 0);
  return C;
}

template <int k>
__device__ __forceinline__ void block_step(f4v (&M)[4][4], int lane) {
  diag_inverse(M[k][k], lane);
  const f4v P = M[k][k];
  f4v O[4];
#pragma unroll
  for (int J = 0; J < 4; ++J) O[J] = M[k][J];
  f4v T[4];
#pragma unroll
  for (int J = 0; J < 4; ++J)
    if (J != k) T[J] = mm(P, O[J], (f4v)(0.0f));
  // rows processed before k: M_Ik = -O_I^T, so M_IJ -= M_Ik T_J = + O_I^T T_J
#pragma unroll
  for (int I = 0; I < k; ++I) {
#pragma unroll
    for (int J = 0; J < 4; ++J)
      if (J != k) M[I][J] = mm(O[I], T[J], M[I][J]);
    M[I][k] = mm(O[I], P, (f4v)(0.0f));  // -M_Ik P = O_I^T P
  }
  // rows after k: M_Ik = +O_I^T
#pragma unroll
  for (int J = 0; J < 4; ++J)
    if (J != k) T[J] = -T[J];
  const f4v nP = -P;
#pragma unroll
  for (int I = k + 1; I < 4; ++I) {
#pragma unroll
    for (int J = 0; J < 4; ++J)
      if (J != k) M[I][J] = mm(O[I], T[J], M[I][J]);
    M[I][k] = mm(O[I], nP, (f4v)(0.0f));
  }
#pragma unroll
  for (int J = 0; J < 4; ++J)
    if (J != k) M[k][J] = -T[J];
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void gj_mfma(const float *in, float *out, int reps) {
  __shared__ __attribute__((aligned(16))) float sc[64][20];
  const int t = threadIdx.x, lane = t;
  const int64_t b = blockIdx.x;
  const int j = lane & 15, g = lane >> 4;
  float K[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) K[c] = in[(b & 255) * 4096 + t * 64 + c];
  for (int rep = 0; rep < reps; ++rep) {
    f4v M[4][4];
    // row layout -> C layout, one 16-column chunk at a time (symmetric input:
    // M[16I+4g+r][16J+j] = row 16J+j, columns 16I+4g..+3)
#pragma unroll
    for (int I = 0; I < 4; ++I) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f4v *>(&sc[t][4 * q]) = (f4v){K[16 * I + 4 * q], K[16 * I + 4 * q + 1], K[16 * I + 4 * q + 2], K[16 * I + 4 * q + 3]};
      wsync();
#pragma unroll
      for (int J = 0; J < 4; ++J) M[I][J] = *reinterpret_cast<const f4v *>(&sc[16 * J + j][4 * g]);
      wsync();
    }
    block_step<0>(M, lane);
    block_step<1>(M, lane);
    block_step<2>(M, lane);
    block_step<3>(M, lane);
    // C layout -> row layout (the inverse is symmetric as well)
#pragma unroll
    for (int I = 0; I < 4; ++I) {
#pragma unroll
      for (int J = 0; J < 4; ++J) *reinterpret_cast<f4v *>(&sc[16 * J + j][4 * g]) = M[I][J];
      wsync();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4v v = *reinterpret_cast<const f4v *>(&sc[t][4 * q]);
        K[16 * I + 4 * q] = v.x;
        K[16 * I + 4 * q + 1] = v.y;
        K[16 * I + 4 * q + 2] = v.z;
        K[16 * I + 4 * q + 3] = v.w;
      }
      wsync();
    }
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) out[b * 4096 + t * 64 + c] = K[c];
}

static void ref_inverse(const std::vector<double> &A, std::vector<double> &X) {
  const int n = 64;
  std::vector<double> M(A);
  X.assign(n * n, 0.0);
  for (int i = 0; i < n; ++i) X[i * n + i] = 1.0;
  for (int k = 0; k < n; ++k) {
    const double p = M[k * n + k];
    for (int c = 0; c < n; ++c) {
      M[k * n + c] /= p;
      X[k * n + c] /= p;
    }
    for (int r = 0; r < n; ++r)
      if (r != k) {
        const double f = M[r * n + k];
        for (int c = 0; c < n; ++c) {
          M[r * n + c] -= f * M[k * n + c];
          X[r * n + c] -= f * X[k * n + c];
        }
      }
  }
}

int main() {
  const int NM = 256, n = 60;
  std::vector<float> hA((size_t)NM * 4096);
  std::vector<std::vector<double>> ref(NM);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; };
  for (int m = 0; m < NM; ++m) {
    // SPD: B B^T / n + diag, equilibrated-looking (O(1) diagonal)
    std::vector<double> Bm(n * n), A(64 * 64, 0.0);
    for (auto &v : Bm) v = rnd();
    for (int i = 0; i < n; ++i)
      for (int jj = 0; jj < n; ++jj) {
        double acc = 0;
        for (int q = 0; q < n; ++q) acc += Bm[i * n + q] * Bm[jj * n + q];
        A[i * 64 + jj] = acc / n * 3.0 + (i == jj ? 0.05 : 0.0);
      }
    for (int i = n; i < 64; ++i) A[i * 64 + i] = 1.0;
    for (int i = 0; i < 4096; ++i) hA[(size_t)m * 4096 + i] = (float)A[i];
    std::vector<double> Af(4096);
    for (int i = 0; i < 4096; ++i) Af[i] = hA[(size_t)m * 4096 + i];
    ref_inverse(Af, ref[m]);
  }
  float *dA, *dO;
  const int BMAX = 16384;
  hipMalloc(&dA, hA.size() * 4);
  hipMalloc(&dO, (size_t)BMAX * 4096 * 4);
  hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
  std::vector<float> hO((size_t)NM * 4096);
  for (int form = 0; form < 2; ++form) {
    auto launch = [&](int B, int reps) {
      if (form == 0)
        hipLaunchKernelGGL(gj_dpp, dim3(B), dim3(64), 0, 0, dA, dO, reps);
      else
        hipLaunchKernelGGL(gj_mfma, dim3(B), dim3(64), 0, 0, dA, dO, reps);
    };
    launch(NM, 1);
    hipDeviceSynchronize();
    hipMemcpy(hO.data(), dO, hO.size() * 4, hipMemcpyDeviceToHost);
    double maxrel = 0;
    for (int m = 0; m < NM; ++m) {
      double num = 0, den = 0;
      for (int i = 0; i < 4096; ++i) {
        num = fmax(num, fabs(hO[(size_t)m * 4096 + i] - ref[m][i]));
        den = fmax(den, fabs(ref[m][i]));
      }
      maxrel = fmax(maxrel, num / den);
    }
    printf("%s: max |X - X_ref| / max|X_ref| = %.3e\n", form ? "mfma" : "dpp ", maxrel);
    for (int B : {1, 1024, 2048, 4096, 8192, 16384}) {
      const int reps = 20;
      launch(B, reps);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      launch(B, reps);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      printf("  %s B %6d  %8.2f us per inverse round  (%.1f cycles @2.4GHz per wave-inverse at this load)\n",
             form ? "mfma" : "dpp ", B, us, us * 2.4e3 / ((B + 1023) / 1024));
    }
  }
  return 0;
}
