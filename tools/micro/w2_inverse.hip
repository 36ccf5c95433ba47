// Probe: the two-wave SRBD KKT inverses (register-row DPP Gauss-Jordan
// invert_w2 vs the matrix-core block Gauss-Jordan invert_w2_mfma) on SPD
// matrices with the W = 2 row layout (wave w, lane v: row 64w + v, 128
// columns; column 63 and columns >= 64 + ncol1 are padding with a diagonal
// only).  Reports max |K X - I| for each form and condition-number band.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -mllvm
//   -pragma-unroll-threshold=200000 -I../../include -I../../quadrupedal_loco_amd/csrc
//   w2_inverse.hip -o w2_inverse
#include "qloco_srbd.hip"
#include "srbd_mfma_inverse.inc"
namespace qloco {
void set_last_error(const char *, hipError_t) {}
}  // probe: the C-ABI error slot lives in qloco_capi.hip

#include <cmath>
#include <cstdio>
#include <vector>

using namespace qloco;

template <bool MF>
__global__ __launch_bounds__(64) void inv1_kernel(const float *in, float *out, const int *ncols) {
  __shared__ __attribute__((aligned(16))) SrbdLds<1> S;
  __shared__ __attribute__((aligned(16))) float sc[16 * 68];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  Row<1> K;
#pragma unroll
  for (int c = 0; c < 64; ++c) K.k[c] = in[b * 16384 + t * 128 + c];
  if constexpr (MF) {
    invert_w1_mfma(sc, t, ncols[b], K);
  } else {
    invert_w1<false>(S, t, ncols[b], K);
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) out[b * 16384 + t * 128 + c] = K.k[c];
}

template <bool MF>
__global__ __launch_bounds__(128) void inv_kernel(const float *in, float *out, const int *ncol1s) {
  __shared__ __attribute__((aligned(16))) SrbdLds<2> S;
  __shared__ __attribute__((aligned(16))) float sc[2 * 8 * 256];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  Row<2> K;
#pragma unroll
  for (int c = 0; c < 128; ++c) K.k[c] = in[b * 16384 + t * 128 + c];
  const int n1 = ncol1s[b];
  if constexpr (MF) {
    invert_w2_mfma(sc, t, n1, K);
  } else {
    const int ncol[2] = {63, n1};
    invert_w2(S, t, ncol, half2_chunks(n1), K);
  }
#pragma unroll
  for (int c = 0; c < 128; ++c) out[b * 16384 + t * 128 + c] = K.k[c];
}

static int run(bool W1) {
  const int NM = 96;  // 6 condition bands of 16
  std::vector<float> hK((size_t)NM * 16384, 0.0f);
  std::vector<int> n1s(NM);
  unsigned s = 777;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; };
  std::vector<std::vector<double>> Kd(NM);
  for (int m = 0; m < NM; ++m) {
    const int n1 = W1 ? 3 * (1 + (m % 20)) : 3 + 3 * (m % 21);  // valid columns (W1: of 60)
    n1s[m] = n1;
    std::vector<int> idx;
    if (W1) {
      for (int c = 0; c < n1; ++c) idx.push_back(c);
    } else {
      for (int c = 0; c < 63; ++c) idx.push_back(c);
      for (int c = 0; c < n1; ++c) idx.push_back(64 + c);
    }
    const int n = idx.size();
    // SPD with eigenvalues spread over 10^(m/16) decades
    const double decades = 1.0 + (m / 16);  // 1e1 .. 1e6
    std::vector<double> Q(n * n);
    for (auto &v : Q) v = rnd();
    // Gram-Schmidt
    for (int i = 0; i < n; ++i) {
      for (int j = 0; j < i; ++j) {
        double d = 0;
        for (int k = 0; k < n; ++k) d += Q[i * n + k] * Q[j * n + k];
        for (int k = 0; k < n; ++k) Q[i * n + k] -= d * Q[j * n + k];
      }
      double nr = 0;
      for (int k = 0; k < n; ++k) nr += Q[i * n + k] * Q[i * n + k];
      nr = sqrt(nr);
      for (int k = 0; k < n; ++k) Q[i * n + k] /= nr;
    }
    std::vector<double> A(128 * 128, 0.0);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double acc = 0;
        for (int k = 0; k < n; ++k) acc += Q[k * n + i] * Q[k * n + j] * pow(10.0, -decades * k / (n - 1));
        A[idx[i] * 128 + idx[j]] = acc;
      }
    for (int c = 0; c < (W1 ? 64 : 128); ++c)
      if (A[c * 128 + c] == 0.0) A[c * 128 + c] = 3.0;  // padding diagonal
    Kd[m].resize(16384);
    for (int i = 0; i < 16384; ++i) {
      hK[(size_t)m * 16384 + i] = (float)A[i];
      Kd[m][i] = (float)A[i];
    }
  }
  float *dK, *dO;
  int *dn;
  (void)hipMalloc(&dK, hK.size() * 4);
  (void)hipMalloc(&dO, hK.size() * 4);
  (void)hipMalloc(&dn, NM * 4);
  (void)hipMemcpy(dK, hK.data(), hK.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dn, n1s.data(), NM * 4, hipMemcpyHostToDevice);
  std::vector<float> hO(hK.size());
  for (int form = 0; form < 2; ++form) {
    if (W1) {
      if (form)
        hipLaunchKernelGGL(inv1_kernel<true>, dim3(NM), dim3(64), 0, 0, dK, dO, dn);
      else
        hipLaunchKernelGGL(inv1_kernel<false>, dim3(NM), dim3(64), 0, 0, dK, dO, dn);
    } else {
      if (form)
        hipLaunchKernelGGL(inv_kernel<true>, dim3(NM), dim3(128), 0, 0, dK, dO, dn);
      else
        hipLaunchKernelGGL(inv_kernel<false>, dim3(NM), dim3(128), 0, 0, dK, dO, dn);
    }
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(hO.data(), dO, hO.size() * 4, hipMemcpyDeviceToHost);
    for (int band = 0; band < 6; ++band) {
      double worst = 0;
      int wm = -1;
      for (int m = band * 16; m < band * 16 + 16; ++m) {
        // residual K X - I over the valid index set (padding rows excluded)
        double r = 0;
        for (int i = 0; i < 128; ++i) {
          if (W1 ? i >= n1s[m] : (i == 63 || i >= 64 + n1s[m])) continue;
          for (int j = 0; j < 128; ++j) {
            if (W1 ? j >= n1s[m] : (j == 63 || j >= 64 + n1s[m])) continue;
            double acc = 0;
            for (int k = 0; k < 128; ++k) acc += Kd[m][i * 128 + k] * hO[(size_t)m * 16384 + k * 128 + j];
            r = fmax(r, fabs(acc - (i == j ? 1.0 : 0.0)));
          }
        }
        if (r > worst) {
          worst = r;
          wm = m;
        }
      }
      printf("W=%d %s cond ~1e%d: max |K X - I| = %.3e (matrix %d, ncol1 %d)\n", W1 ? 1 : 2, form ? "mfma" : "dpp ",
             band + 1, worst, wm, wm >= 0 ? n1s[wm] : -1);
    }
  }
  return 0;
}

int main() {
  run(true);
  run(false);
  return 0;
}
