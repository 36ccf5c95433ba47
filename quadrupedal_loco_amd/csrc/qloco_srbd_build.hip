// qloco_srbd_build.hip -- batched dense condensed-QP build (the literal
// matrices ConvexMpc::calculate_qp_mats materialises,
// a1_cpp_open_source/src/ConvexMpc.cpp:162-264, with the compute_grf
// inputs of A1RobotControl.cpp:452-549), for callers that want A_qp, B_qp,
// H, g, lb, ub themselves (e.g. to feed another QP solver).  The fused
// solve path (qloco_srbd.hip) never materialises these.
//
// One workgroup (256 threads) per instance.  The per-step B_d and
// E = dt A_c B_d blocks live in LDS; every output entry is an independent
// closed form (A_c^3 = 0, A_c^2 B_d = 0, see qloco_srbd.hip), written with
// consecutive threads on consecutive column-major addresses.  The kernel is
// bound by the HBM write of H ((12N)^2 floats per instance).
#include <math.h>
#include <string.h>

#include "qloco_common.hpp"

namespace qloco {

constexpr int kBuildMaxN = 20;

struct BuildArgs {
  int N, feet_per_step, contacts_per_step;
  float dt, mass, mu, fz_min, fz_max;
  float inertia[9];
  float q2[13], r2[12];
  int64_t batch;
  const float *x0, *xref, *feet;
  const uint8_t *contacts;
  float *H, *g, *lb, *ub, *Aqp, *Bqp;
};

__global__ __launch_bounds__(256) void srbd_build_kernel(const BuildArgs a) {
  __shared__ float Bd[kBuildMaxN][6][12];  // rows 6..11 of B_d (rows 0..5 are zero)
  __shared__ float Ed[kBuildMaxN][6][12];  // rows 0..5 of E = dt A_c B_d
  __shared__ float q2[13];
  __shared__ float r2[12];
  __shared__ float x0[13];
  __shared__ float werr[kBuildMaxN * 13];  // Q (Aqp x0 - x_ref)
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int N = a.N, nx = 13 * N, nu = 12 * N, nc = 20 * N;
  const float dt = a.dt;
  if (t == 0) {
#pragma unroll
    for (int k = 0; k < 13; ++k) q2[k] = a.q2[k];
#pragma unroll
    for (int k = 0; k < 12; ++k) r2[k] = a.r2[k];
  }
  if (t < 13) x0[t] = a.x0[b * 13 + t];
  __syncthreads();
  const float yaw = x0[2];
  const float cy = cosf(yaw), sy = sinf(yaw);
  // yaw "rotation" overwriting root_rot_mat (A1RobotControl.cpp:502-510)
  const float Rm[3][3] = {{cy, sy, 0.f}, {-sy, cy, 0.f}, {0.f, 0.f, 1.f}};
  // B_c (ConvexMpc.cpp:135-147): rows 6..8 = I_w^-1 skew(r_i), rows 9..11 = I/m
  for (int idx = t; idx < N * 12; idx += 256) {
    const int k = idx / 12, col = idx - 12 * k;
    const int leg = col / 3, comp = col - 3 * leg;
    float RI[3][3], Iw[3][3], Ii[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        RI[r][c] = Rm[r][0] * a.inertia[c * 3 + 0] + Rm[r][1] * a.inertia[c * 3 + 1] +
                   Rm[r][2] * a.inertia[c * 3 + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        Iw[r][c] = RI[r][0] * Rm[c][0] + RI[r][1] * Rm[c][1] + RI[r][2] * Rm[c][2];
    const float c00 = Iw[1][1] * Iw[2][2] - Iw[1][2] * Iw[2][1];
    const float c01 = Iw[1][2] * Iw[2][0] - Iw[1][0] * Iw[2][2];
    const float c02 = Iw[1][0] * Iw[2][1] - Iw[1][1] * Iw[2][0];
    const float id = 1.0f / (Iw[0][0] * c00 + Iw[0][1] * c01 + Iw[0][2] * c02);
    Ii[0][0] = c00 * id;
    Ii[1][0] = c01 * id;
    Ii[2][0] = c02 * id;
    Ii[0][1] = (Iw[0][2] * Iw[2][1] - Iw[0][1] * Iw[2][2]) * id;
    Ii[1][1] = (Iw[0][0] * Iw[2][2] - Iw[0][2] * Iw[2][0]) * id;
    Ii[2][1] = (Iw[0][1] * Iw[2][0] - Iw[0][0] * Iw[2][1]) * id;
    Ii[0][2] = (Iw[0][1] * Iw[1][2] - Iw[0][2] * Iw[1][1]) * id;
    Ii[1][2] = (Iw[0][2] * Iw[1][0] - Iw[0][0] * Iw[1][2]) * id;
    Ii[2][2] = (Iw[0][0] * Iw[1][1] - Iw[0][1] * Iw[1][0]) * id;
    const float *rf = a.feet + b * (a.feet_per_step ? nu : 12) + (a.feet_per_step ? 12 * k : 0) + 3 * leg;
    const float rx = rf[0], ry = rf[1], rz = rf[2];
    const float tv0 = comp == 0 ? 0.f : (comp == 1 ? -rz : ry);  // skew(r) e_comp (Utils.cpp:35-41)
    const float tv1 = comp == 0 ? rz : (comp == 1 ? 0.f : -rx);
    const float tv2 = comp == 0 ? -ry : (comp == 1 ? rx : 0.f);
    float w[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) w[r] = dt * (Ii[r][0] * tv0 + Ii[r][1] * tv1 + Ii[r][2] * tv2);
    const float vm = dt / a.mass;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      Bd[k][r][col] = w[r];
      Bd[k][3 + r][col] = (r == comp) ? vm : 0.0f;
    }
    // E = dt A_c B_d: rows 0..2 = dt Rz w, rows 3..5 = dt v-rows
    Ed[k][0][col] = dt * (Rm[0][0] * w[0] + Rm[0][1] * w[1]);
    Ed[k][1][col] = dt * (Rm[1][0] * w[0] + Rm[1][1] * w[1]);
    Ed[k][2][col] = dt * w[2];
#pragma unroll
    for (int r = 0; r < 3; ++r) Ed[k][3 + r][col] = (r == comp) ? dt * vm : 0.0f;
  }
  // Q (A_qp x0 - x_ref), free response in closed form
  for (int idx = t; idx < nx; idx += 256) {
    const int i = idx / 13, s = idx - 13 * i;
    const float k = (float)(i + 1);
    float xf;
    if (s < 3) {
      const float rw = s == 0 ? (cy * x0[6] + sy * x0[7]) : (s == 1 ? (-sy * x0[6] + cy * x0[7]) : x0[8]);
      xf = x0[s] + k * dt * rw;
    } else if (s < 6) {
      xf = x0[s] + k * dt * x0[s + 6];
      if (s == 5) xf += 0.5f * k * (k - 1.0f) * dt * dt * x0[12];
    } else if (s < 9) {
      xf = x0[s];
    } else if (s < 12) {
      xf = x0[s] + (s == 11 ? k * dt * x0[12] : 0.0f);
    } else {
      xf = x0[12];
    }
    werr[idx] = q2[s] * (xf - a.xref[b * nx + idx]);
  }
  __syncthreads();

  // H = B_qp' Q B_qp + R (ConvexMpc.cpp:207-215), col-major, closed form
  if (a.H) {
    float *H = a.H + b * (int64_t)nu * nu;
    for (int idx = t; idx < nu * nu; idx += 256) {
      const int c = idx / nu, r = idx - c * nu;
      const int jr = r / 12, ar = r - 12 * jr, jc = c / 12, ac = c - 12 * jc;
      const int M = jr > jc ? jr : jc;
      const int T = N - M, al = M - jr, be = M - jc;
      const float K0 = (float)T;
      const float K2 = (float)((T - 1) * T * (2 * T - 1) / 6 + (al + be) * (T * (T - 1) / 2) + al * be * T);
      float bb = 0.f, ee = 0.f;
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        bb += Bd[jr][s][ar] * q2[6 + s] * Bd[jc][s][ac];
        ee += Ed[jr][s][ar] * q2[s] * Ed[jc][s][ac];
      }
      float h = K0 * bb + K2 * ee;
      if (r == c) h += r2[ar];
      H[idx] = h;
    }
  }
  // g = B_qp' Q (A_qp x0 - x_ref) (:219-221)
  if (a.g) {
    for (int c = t; c < nu; c += 256) {
      const int jc = c / 12, ac = c - 12 * jc;
      float acc = 0.f;
      for (int i = jc; i < N; ++i) {
        const float kk = (float)(i - jc);
#pragma unroll
        for (int s = 0; s < 6; ++s)
          acc += (Bd[jc][s][ac] * werr[13 * i + 6 + s] + kk * Ed[jc][s][ac] * werr[13 * i + s]);
      }
      a.g[b * nu + c] = acc;
    }
  }
  // bounds (:223-249), fz_min / fz_max scaled by the contact flag
  if (a.lb && a.ub) {
    const int nct = a.contacts_per_step ? 4 * N : 4;
    for (int idx = t; idx < nc; idx += 256) {
      const int k = idx / 20, w = idx - 20 * k, leg = w / 5, row = w - 5 * leg;
      const float cf = a.contacts[b * nct + (a.contacts_per_step ? 4 * k + leg : leg)] ? 1.0f : 0.0f;
      const float lo[5] = {0.f, -1e30f, 0.f, -1e30f, a.fz_min * cf};
      const float hi[5] = {1e30f, 0.f, 1e30f, 0.f, a.fz_max * cf};
      a.lb[b * nc + idx] = lo[row];
      a.ub[b * nc + idx] = hi[row];
    }
  }
  // A_qp block i = A_d^{i+1} = I + k dt A_c + k(k-1)/2 dt^2 A_c^2 (:188-195)
  if (a.Aqp) {
    float *A = a.Aqp + b * (int64_t)nx * 13;
    for (int idx = t; idx < nx * 13; idx += 256) {
      const int col = idx / nx, row = idx - col * nx;
      const int i = row / 13, s = row - 13 * i;
      const float k = (float)(i + 1);
      float v = (s == col) ? 1.0f : 0.0f;
      // A_c entries
      float ac = 0.f;
      if (s < 3 && col >= 6 && col < 9) ac = Rm[s][col - 6];
      if (s >= 3 && s < 6 && col == s + 6) ac = 1.0f;
      if (s == 11 && col == 12) ac = 1.0f;
      // A_c^2 entries: p_z <- gravity
      const float ac2 = (s == 5 && col == 12) ? 1.0f : 0.0f;
      v += k * dt * ac + 0.5f * k * (k - 1.0f) * dt * dt * ac2;
      A[idx] = v;
    }
  }
  // B_qp block (i, j <= i) = A_d^{i-j} B_d,j = B_d,j + (i-j) E_j (:196-205)
  if (a.Bqp) {
    float *Bq = a.Bqp + b * (int64_t)nx * nu;
    for (int idx = t; idx < nx * nu; idx += 256) {
      const int col = idx / nx, row = idx - col * nx;
      const int i = row / 13, s = row - 13 * i, j = col / 12, cc = col - 12 * j;
      float v = 0.f;
      if (i >= j && s < 12) v = (s >= 6) ? Bd[j][s - 6][cc] : (float)(i - j) * Ed[j][s][cc];
      Bq[idx] = v;
    }
  }
}

}  // namespace qloco

using namespace qloco;

extern "C" int qloco_srbd_build(const qloco_srbd_spec *spec, int64_t batch, const float *x0,
                                const float *x_ref, const float *feet, const uint8_t *contacts,
                                float *H, float *g, float *lb, float *ub, float *Aqp, float *Bqp,
                                void *stream) {
  if (!spec || batch < 0) return QLOCO_ERR_ARG;
  if (spec->horizon < 1 || spec->horizon > kBuildMaxN) return QLOCO_BAD_SIZE;
  if (batch == 0) return QLOCO_OK;
  if (!x0 || !x_ref || !feet) return QLOCO_ERR_ARG;
  if ((lb || ub) && (!lb || !ub || !contacts)) return QLOCO_ERR_ARG;
  if (spec->mass <= 0.0f || spec->dt <= 0.0f) return QLOCO_ERR_ARG;
  BuildArgs a;
  memset(&a, 0, sizeof(a));
  a.N = spec->horizon;
  a.feet_per_step = spec->feet_per_step;
  a.contacts_per_step = spec->contacts_per_step;
  a.dt = spec->dt;
  a.mass = spec->mass;
  a.mu = spec->mu;
  a.fz_min = spec->fz_min;
  a.fz_max = spec->fz_max;
  for (int k = 0; k < 9; ++k) a.inertia[k] = spec->inertia[k];
  for (int k = 0; k < 13; ++k) a.q2[k] = 2.0f * spec->q_weights[k];
  for (int k = 0; k < 12; ++k) a.r2[k] = 2.0f * spec->r_weights[k];
  a.batch = batch;
  a.x0 = x0;
  a.xref = x_ref;
  a.feet = feet;
  a.contacts = contacts;
  a.H = H;
  a.g = g;
  a.lb = lb;
  a.ub = ub;
  a.Aqp = Aqp;
  a.Bqp = Bqp;
  hipLaunchKernelGGL(srbd_build_kernel, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "srbd_build_kernel launch");
  return QLOCO_OK;
}
