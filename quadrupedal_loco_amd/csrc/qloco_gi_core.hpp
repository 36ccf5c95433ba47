// qloco_gi_core.hpp -- Goldfarb-Idnani dual active-set QP, one instance per
// 16-lane group (device code shared by qloco_gi.hip, qloco_force.hip and
// qloco_body.hip).  See qloco_gi.hip for the design notes.  Translation
// units that include this header must be compiled with -ffp-contract=off.
#pragma once
#include <float.h>
#include <math.h>

#include "qloco_common.hpp"

namespace qloco {

constexpr int GI_N = 16;                 // max variables
constexpr int GI_P = 16;                 // max equalities
constexpr int GI_M = 64;                 // max inequalities
constexpr int GI_PM = GI_P + GI_M + 1;
constexpr int GI_GROUPS = 4;             // instances per wavefront

// Per-group LDS work space, sized for at most NN variables, MM inequalities
// and PP equalities (the generic kernel uses the GI_* limits; the force and
// body kernels instantiate their exact sizes so more groups fit per CU).
// The active set never holds more than max(n, p) + 1 entries (equality i is
// recorded at index i < p, the quirk of EiQuadProg.cpp:268; inequalities at
// iq <= n), so A/u/r are sized AS; iai/iaexcl are indexed by constraint.
template <int NN, int MM, int PP>
struct GiLdsT {
  static constexpr int AS = (NN > PP ? NN : PP) + 1;
  double J[NN * NN];  // col-major, J(r,c) = J[c*NN + r]
  double R[NN * NN];
  double x[NN], z[NN], d[NN], np[NN], xold[NN];
  double s[MM];
  double r[AS], u[AS], uold[AS];
  int A[AS], Aold[AS], iai[MM], iaexcl[MM];
};
using GiLds = GiLdsT<GI_N, GI_M, GI_P>;

struct GiArgs {
  int n, p, m;
  int64_t batch;
  const double *G, *g0, *CE, *ce0, *CI, *ci0;
  int64_t sG, sg0, sCE, sce0, sCI, sci0;
  double *x, *f;
  int *status, *iters;
};

#define GI_SYNC() asm volatile("" ::: "memory")

// Development-only phase clocks of the solve (tools/gi_phase.py builds a
// variant library with -DQLOCO_GI_PHASE_TIMING; the product never defines it)
#ifdef QLOCO_GI_PHASE_TIMING
static __device__ unsigned int g_gi_phase[(1 << 16) * 8];
#define GI_PHASE(i)                                                                   \
  do {                                                                                \
    const uint64_t _n = __builtin_readcyclecounter();                                 \
    const int64_t _g = (int64_t)blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);  \
    if (li == 0 && _g < (1 << 16)) g_gi_phase[_g * 8 + (i)] = (unsigned)(_n - _gt0);   \
  } while (0)
#define GI_STAMP(v) const uint64_t v = __builtin_readcyclecounter()
#define GI_ACC(i, v0)                                                                 \
  do {                                                                                \
    const uint64_t _n = __builtin_readcyclecounter();                                 \
    const int64_t _g = (int64_t)blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);  \
    if (li == 0 && _g < (1 << 16)) g_gi_phase[_g * 8 + (i)] += (unsigned)(_n - (v0)); \
  } while (0)
#else
#define GI_PHASE(i) ((void)0)
#define GI_STAMP(v) ((void)0)
#define GI_ACC(i, v0) ((void)0)
#endif

__device__ __forceinline__ double gi_distance(double a, double b) {  // EiQuadProg.hpp:100-118
  const double a1 = fabs(a), b1 = fabs(b);
  double t;
  if (a1 > b1) {
    t = b1 / a1;
    return a1 * sqrt(1.0 + t * t);
  }
  if (b1 > a1) {
    t = a1 / b1;
    return b1 * sqrt(1.0 + t * t);
  }
  return a1 * sqrt(2.0);
}

// One group's view of the problem.
template <int NN, int MM, int PP>
struct GiGroup {
  GiLdsT<NN, MM, PP> *L;
  int li;  // lane in group (0..15)
  int n, p, m;
  const double *CE, *ce0, *CI, *ci0;
  __device__ __forceinline__ double J(int r, int c) const { return L->J[c * NN + r]; }
  __device__ __forceinline__ double &Jr(int r, int c) { return L->J[c * NN + r]; }
  __device__ __forceinline__ double &Rr(int r, int c) { return L->R[c * NN + r]; }
  __device__ __forceinline__ double CEc(int r, int i) const { return CE[(int64_t)i * n + r]; }
  __device__ __forceinline__ double CIc(int r, int i) const { return CI[(int64_t)i * n + r]; }

  // d = J' np : lane c sums its column in row order
  __device__ __forceinline__ void compute_d() {
    const int c = li;
    if (c < n) {
      double acc = 0.0;
      for (int r = 0; r < n; ++r) acc += J(r, c) * L->np[r];
      L->d[c] = acc;
    }
    GI_SYNC();
  }
  // z = J(:, iq:) d(iq:) : lane r sums its row in column order
  __device__ __forceinline__ void update_z(int iq) {
    const int r = li;
    if (r < n) {
      double acc = 0.0;
      for (int c = iq; c < n; ++c) acc += J(r, c) * L->d[c];
      L->z[r] = acc;
    }
    GI_SYNC();
  }
  // r(0:iq) = triu(R)^-1 d(0:iq) : back substitution, every lane the same
  // operations in the same order, the solved entries carried in registers
  // (the pass unrolled over the NN possible rows: static register indices),
  // the R / d reads independent of the chain; lane 0 stores r at the end.
  __device__ __forceinline__ void update_r(int iq) {
    double rv[NN];
#pragma unroll
    for (int i = NN - 1; i >= 0; --i) {
      rv[i] = 0.0;
      if (i >= iq) continue;
      double acc = L->d[i];
#pragma unroll
      for (int j = i + 1; j < NN; ++j)
        if (j < iq) acc -= L->R[j * NN + i] * rv[j];
      rv[i] = acc / L->R[i * NN + i];
    }
    GI_SYNC();
    if (li == 0) {
#pragma unroll
      for (int i = 0; i < NN; ++i)
        if (i < iq) L->r[i] = rv[i];
    }
    GI_SYNC();
  }
  // EiQuadProg.cpp:30-93 ; returns false when degenerate.  The Givens sweep
  // runs on register copies: d (every lane, identical) and this lane's row
  // of J (lane k: J(k, 0..n-1)); only the stored results go back to LDS.
  __device__ bool add_constraint(int &iq, double &R_norm) {
    double dv[NN], jr[NN];
    const int k = li;
#pragma unroll
    for (int c = 0; c < NN; ++c) {
      dv[c] = L->d[c];
      jr[c] = (k < n) ? J(k, c) : 0.0;
    }
#pragma unroll
    for (int j = NN - 1; j >= 1; j--) {
      if (j > n - 1 || j < iq + 1) continue;
      double cc = dv[j - 1];
      double ss = dv[j];
      const double h = gi_distance(cc, ss);
      if (h == 0.0) continue;
      ss = ss / h;
      cc = cc / h;
      double dj1;
      if (cc < 0.0) {
        cc = -cc;
        ss = -ss;
        dj1 = -h;
      } else {
        dj1 = h;
      }
      dv[j] = 0.0;
      dv[j - 1] = dj1;
      const double xny = ss / (1.0 + cc);
      const double t1 = jr[j - 1];
      const double t2 = jr[j];
      const double nj1 = t1 * cc + t2 * ss;
      jr[j - 1] = nj1;
      jr[j] = xny * (t1 + nj1) - t2;
    }
    GI_SYNC();
    if (li == 0) {
#pragma unroll
      for (int c = 0; c < NN; ++c) L->d[c] = dv[c];
    }
    if (k < n) {
#pragma unroll
      for (int c = 0; c < NN; ++c)
        if (c < n) Jr(k, c) = jr[c];
    }
    GI_SYNC();
    iq++;
    if (li < iq) Rr(li, iq - 1) = L->d[li];
    GI_SYNC();
    const double dl = fabs(L->d[iq - 1]);
    if (dl <= DBL_EPSILON * R_norm) return false;
    if (dl > R_norm) R_norm = dl;
    return true;
  }
  // EiQuadProg.cpp:95-170 ; returns false on the reference's UB path
  __device__ bool delete_constraint(int p_, int &iq, int l) {
    int qq = -1;
    for (int i = p_; i < iq; i++)
      if (L->A[i] == l) {
        qq = i;
        break;
      }
    if (qq < 0) return false;
    // shift A / u / the R columns qq+1..iq-1 one place left: every value
    // read before any is written (pure moves, the reference's result)
    {
      int a_n[2] = {0, 0};
      double u_n[2] = {0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = qq + li + 16 * q;
        if (i < iq - 1) {
          a_n[q] = L->A[i + 1];
          u_n[q] = L->u[i + 1];
        }
      }
      double rcol[NN];
#pragma unroll
      for (int i = 0; i < NN; ++i) rcol[i] = (li < n && i >= qq && i < iq - 1) ? L->R[(i + 1) * NN + li] : 0.0;
      GI_SYNC();
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = qq + li + 16 * q;
        if (i < iq - 1) {
          L->A[i] = a_n[q];
          L->u[i] = u_n[q];
        }
      }
#pragma unroll
      for (int i = 0; i < NN; ++i)
        if (li < n && i >= qq && i < iq - 1) Rr(li, i) = rcol[i];
    }
    GI_SYNC();
    if (li == 0) {
      L->A[iq - 1] = L->A[iq];
      L->u[iq - 1] = L->u[iq];
      L->A[iq] = 0;
      L->u[iq] = 0.0;
    }
    if (li < iq) Rr(li, iq - 1) = 0.0;
    GI_SYNC();
    iq--;
    if (iq == 0) return true;
    for (int j = qq; j < iq; j++) {
      double cc = L->R[j * NN + j];
      double ss = L->R[j * NN + j + 1];
      const double h = gi_distance(cc, ss);
      if (h == 0.0) continue;
      cc = cc / h;
      ss = ss / h;
      double rjj;
      if (cc < 0.0) {
        rjj = -h;
        cc = -cc;
        ss = -ss;
      } else {
        rjj = h;
      }
      const double xny = ss / (1.0 + cc);
      GI_SYNC();
      if (li == 0) {
        Rr(j + 1, j) = 0.0;
        Rr(j, j) = rjj;
      }
      // rows j, j+1 of R over columns k = j+1 .. iq-1 : lane k
      {
        const int k = li;
        if (k >= j + 1 && k < iq) {
          const double t1 = L->R[k * NN + j];
          const double t2 = L->R[k * NN + j + 1];
          const double nj = t1 * cc + t2 * ss;
          Rr(j, k) = nj;
          Rr(j + 1, k) = xny * (t1 + nj) - t2;
        }
      }
      // columns j, j+1 of J : lane = row
      {
        const int k = li;
        if (k < n) {
          const double t1 = J(k, j);
          const double t2 = J(k, j + 1);
          const double nj = t1 * cc + t2 * ss;
          Jr(k, j) = nj;
          Jr(k, j + 1) = xny * (nj + t1) - t2;
        }
      }
      GI_SYNC();
    }
    return true;
  }
};

// Solve one QP with the 16 lanes of a group.  G (n x n, ld = ldG), g0, CE
// (n x p), ce0, CI (n x m), ci0 may live in global memory or LDS (flat
// pointers).  Writes x (n) to xout (lane li < n writes element li).
template <int NN, int MM, int PP>
__device__ __forceinline__ void gi_solve_group(GiLdsT<NN, MM, PP> &S, int li, int n, int p, int m, const double *G, int ldG,
                               const double *g0, const double *CE, const double *ce0,
                               const double *CI, const double *ci0, double *xout,
                               double &f_out, int &status_out, int &iters_out) {
  GiGroup<NN, MM, PP> g;
  g.L = &S;
  g.li = li;
  g.n = n;
  g.p = p;
  g.m = m;
  g.CE = CE;
  g.ce0 = ce0;
  g.CI = CI;
  g.ci0 = ci0;
#ifdef QLOCO_GI_PHASE_TIMING
  const uint64_t _gt0 = __builtin_readcyclecounter();
  {
    const int64_t _g = (int64_t)blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);
    if (li == 0 && _g < (1 << 16)) g_gi_phase[_g * 8 + 0] = g_gi_phase[_g * 8 + 6] = g_gi_phase[_g * 8 + 7] = 0;
  }
#endif
  const double inf = INFINITY;
  int status = QLOCO_OK;
  int iter = 0;
  double f_value = 0.0;
  // persistent-member semantics: start every solve from zeroed index arrays
  for (int k = li; k < GiLdsT<NN, MM, PP>::AS; k += 16) {
    S.A[k] = 0;
    S.Aold[k] = 0;
    S.u[k] = 0.0;
    S.r[k] = 0.0;
    S.uold[k] = 0.0;
  }
  for (int k = li; k < MM; k += 16) {
    S.iai[k] = 0;
    S.iaexcl[k] = 0;
  }
  // ---- solve_quadprog: c1 = trace(G); LLT of the lower triangle (EiQuadProg.cpp:493-513)
  double c1 = 0.0;
  for (int i = 0; i < n; ++i) c1 += G[i * ldG + i];
  // L is built in R (zeroed again before solve_quadprog2 uses R).  Only the
  // lower triangle is read before that, so a caller may build G in S.R itself
  // (ldG = NN): the copy below is then in place and the clear is skipped.
  if (G != S.R)
    for (int k = li; k < NN * NN; k += 16) S.R[k] = 0.0;
  GI_SYNC();
  if (li < n)
    for (int c = 0; c <= li; ++c) S.R[c * NN + li] = G[c * ldG + li];  // lower triangle, row li
  GI_SYNC();
  bool pd = true;
  for (int k = 0; k < n; ++k) {
    double x = S.R[k * NN + k];
    for (int j = 0; j < k; ++j) x -= S.R[j * NN + k] * S.R[j * NN + k];
    if (!(x > 0.0)) {
      pd = false;
      break;
    }
    const double lkk = sqrt(x);
    const int r = li;
    double lrk = 0.0;
    if (r > k && r < n) {
      double acc = S.R[k * NN + r];
      for (int j = 0; j < k; ++j) acc -= S.R[j * NN + r] * S.R[j * NN + k];
      lrk = acc / lkk;
    }
    GI_SYNC();
    if (r > k && r < n) S.R[k * NN + r] = lrk;
    if (li == 0) S.R[k * NN + k] = lkk;
    GI_SYNC();
  }
  GI_PHASE(1);
  if (!pd) {
    status = QLOCO_NOT_PD;
    f_value = inf;
    goto done;
  }
  {
    // J = L^-T : lane c back-substitutes column c (EiQuadProg.cpp:213-214)
    if (li < n) {
      const int c = li;
      for (int rr = n - 1; rr >= 0; --rr) {
        double acc = (rr == c) ? 1.0 : 0.0;
        for (int j = rr + 1; j < n; ++j) acc -= S.R[rr * NN + j] * S.J[c * NN + j];
        S.J[c * NN + rr] = acc / S.R[rr * NN + rr];
      }
    }
    GI_SYNC();
    GI_PHASE(2);
    double c2 = 0.0;
    for (int i = 0; i < n; ++i) c2 += S.J[i * NN + i];
    // x = -G^-1 g0 through the factor (:227-230): every lane the same
    // forward / back substitution in registers (static indices), lane li
    // stores x[li]
    {
      double xv[NN];
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        xv[i] = 0.0;
        if (i >= n) continue;
        double acc = g0[i];
#pragma unroll
        for (int j = 0; j < i; ++j) acc -= S.R[j * NN + i] * xv[j];
        xv[i] = acc / S.R[i * NN + i];
      }
#pragma unroll
      for (int i = NN - 1; i >= 0; --i) {
        if (i >= n) continue;
        double acc = xv[i];
#pragma unroll
        for (int j = i + 1; j < NN; ++j)
          if (j < n) acc -= S.R[i * NN + j] * xv[j];
        xv[i] = acc / S.R[i * NN + i];
      }
      GI_SYNC();
#pragma unroll
      for (int i = 0; i < NN; ++i)
        if (i < n && li == i) S.x[i] = -xv[i];
    }
    GI_SYNC();
    GI_PHASE(3);
    f_value = 0.0;
    for (int i = 0; i < n; ++i) f_value += g0[i] * S.x[i];
    f_value *= 0.5;
    // solve_quadprog2 preprocessing: d = 0, R = 0, R_norm = 1 (:207-209)
    for (int k = li; k < NN * NN; k += 16) S.R[k] = 0.0;
    if (li < NN) S.d[li] = 0.0;
    GI_SYNC();
    double R_norm = 1.0;
    const int me = p, mi = m;
    int iq = 0;
    int ip = 0, l = 0;
    double ss = 0.0, psi, t, t1, t2;

    // ---- equality constraints (:237-276), quirks kept.  The reference
    // skips all-zero CE columns (:239-244); the live columns are found up
    // front (all loads in flight) and the loop runs over them in column
    // order, so the four groups of a wave -- whose swing patterns differ --
    // step through their own live columns together instead of through the
    // union of everyone's.
    {
      unsigned live = 0u;
      for (int i = 0; i < me; i++) {
        bool nz = false;
#pragma unroll
        for (int r = 0; r < NN; ++r)
          if (r < n) nz = nz | (g.CEc(r, i) != 0.0);
        if (nz) live |= 1u << i;
      }
      while (live) {
        const int i = __builtin_ctz(live);
        live &= live - 1u;
        if (li < n) S.np[li] = g.CEc(li, i);
        GI_SYNC();
        g.compute_d();
        g.update_z(iq);
        g.update_r(iq);
        t2 = 0.0;
        double zz = 0.0, znp = 0.0, npx = 0.0;
        for (int k = 0; k < n; ++k) {
          zz += S.z[k] * S.z[k];
          znp += S.z[k] * S.np[k];
          npx += S.np[k] * S.x[k];
        }
        if (fabs(zz) > DBL_EPSILON) t2 = (-npx - g.ce0[i]) / znp;
        GI_SYNC();
        if (li < n) S.x[li] += t2 * S.z[li];
        // u(0:iq) -= t2 r(0:iq): independent entries, one per lane
        for (int k = li; k < iq; k += 16) S.u[k] -= t2 * S.r[k];
        if (li == 0) {
          S.u[iq] = t2;
          S.A[i] = -i - 1;
        }
        GI_SYNC();
        f_value += 0.5 * (t2 * t2) * znp;
        if (!g.add_constraint(iq, R_norm)) {
          status = QLOCO_DEGENERATE;
          goto done;
        }
      }
    }
    for (int i = li; i < mi; i += 16) S.iai[i] = i;
    GI_SYNC();
    GI_PHASE(4);

  l1:
    GI_STAMP(_i0);
    iter++;
    GI_SYNC();
    // active constraints are distinct indices: one store per lane
    for (int i = me + li; i < iq; i += 16) S.iai[S.A[i]] = -1;
    GI_SYNC();
    ss = 0.0;
    psi = 0.0;
    ip = 0;
    // s(x) = CI' x + ci0, one constraint per lane, row order
    for (int i = li; i < mi; i += 16) {
      S.iaexcl[i] = 1;
      double sum = 0.0;
      for (int r = 0; r < n; ++r) sum += g.CIc(r, i) * S.x[r];
      S.s[i] = sum + g.ci0[i];
    }
    GI_SYNC();
    for (int i = 0; i < mi; i++) psi += (S.s[i] < 0.0) ? S.s[i] : 0.0;
    if (fabs(psi) <= mi * DBL_EPSILON * c1 * c2 * 100.0) goto done;
    GI_SYNC();
    for (int i = li; i < iq; i += 16) {
      S.uold[i] = S.u[i];
      S.Aold[i] = S.A[i];
    }
    if (li < n) S.xold[li] = S.x[li];
    GI_SYNC();
    GI_ACC(0, _i0);

  l2:
    for (int i = 0; i < mi; i++) {
      if (S.s[i] < ss && S.iai[i] != -1 && S.iaexcl[i]) {
        ss = S.s[i];
        ip = i;
      }
    }
    if (ss >= 0.0) goto done;
    GI_SYNC();
    if (li < n) S.np[li] = g.CIc(li, ip);
    if (li == 0) {
      S.u[iq] = 0.0;
      S.A[iq] = ip;
    }
    GI_SYNC();

  l2a:
    {
    GI_STAMP(_i1);
    g.compute_d();
    g.update_z(iq);
    g.update_r(iq);
    GI_ACC(6, _i1);
    }
    l = 0;
    t1 = inf;
    for (int k = me; k < iq; k++) {
      double tmp;
      if (S.r[k] > 0.0 && ((tmp = S.u[k] / S.r[k]) < t1)) {
        t1 = tmp;
        l = S.A[k];
      }
    }
    {
      double zz = 0.0, znp = 0.0;
      for (int k = 0; k < n; ++k) {
        zz += S.z[k] * S.z[k];
        znp += S.z[k] * S.np[k];
      }
      if (fabs(zz) > DBL_EPSILON)
        t2 = -S.s[ip] / znp;
      else
        t2 = inf;
      t = (t1 < t2) ? t1 : t2;
      if (t >= inf) {
        status = QLOCO_INFEASIBLE;
        f_value = inf;
        goto done;
      }
      if (t2 >= inf) {
        GI_SYNC();
        for (int k = li; k < iq; k += 16) S.u[k] -= t * S.r[k];
        if (li == 0) {
          S.u[iq] += t;
          S.iai[l] = l;
        }
        GI_SYNC();
        if (!g.delete_constraint(p, iq, l)) {
          status = QLOCO_UB_PATH;
          goto done;
        }
        goto l2a;
      }
      GI_SYNC();
      if (li < n) S.x[li] += t * S.z[li];
      f_value += t * znp * (0.5 * t + S.u[iq]);
      GI_SYNC();
      for (int k = li; k < iq; k += 16) S.u[k] -= t * S.r[k];
      if (li == 0) S.u[iq] += t;
      GI_SYNC();
    }
    if (t == t2) {
      if (!g.add_constraint(iq, R_norm)) {
        GI_SYNC();
        if (li == 0) S.iaexcl[ip] = 0;
        GI_SYNC();
        if (!g.delete_constraint(p, iq, ip)) {
          status = QLOCO_UB_PATH;
          goto done;
        }
        for (int i = li; i < m; i += 16) S.iai[i] = i;
        GI_SYNC();
        bool bad = false;
        for (int i = 0; i < iq; i++) bad = bad || (S.Aold[i] < 0 || S.Aold[i] >= m);
        if (bad) {  // reference: out-of-range write through _iai(_A(i)), UB
          status = QLOCO_UB_PATH;
          goto done;
        }
        if (li == 0)
          for (int i = 0; i < iq; i++) {
            S.A[i] = S.Aold[i];
            S.iai[S.A[i]] = -1;
            S.u[i] = S.uold[i];
          }
        if (li < n) S.x[li] = S.xold[li];
        GI_SYNC();
        goto l2;
      } else {
        GI_SYNC();
        if (li == 0) S.iai[ip] = -1;
        GI_SYNC();
      }
      goto l1;
    }
    // partial step: drop constraint l (:477-490)
    GI_SYNC();
    if (li == 0) S.iai[l] = l;
    GI_SYNC();
    if (!g.delete_constraint(p, iq, l)) {
      status = QLOCO_UB_PATH;
      goto done;
    }
    {
      double sum = 0.0;
      for (int r = 0; r < n; ++r) sum += g.CIc(r, ip) * S.x[r];
      GI_SYNC();
      if (li == 0) S.s[ip] = sum + g.ci0[ip];
      GI_SYNC();
    }
    goto l2a;
  }

done:
  GI_SYNC();
  GI_PHASE(5);
  if (li < n) xout[li] = S.x[li];
  f_out = f_value;
  status_out = status;
  iters_out = iter;
  GI_SYNC();
}

}  // namespace qloco
