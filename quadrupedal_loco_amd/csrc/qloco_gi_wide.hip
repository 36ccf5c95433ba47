// qloco_gi_wide.hip -- Goldfarb-Idnani dual active-set QP for the full
// capacity of the reference's QPBaseClass (nVars <= 60, nIneq <= 300,
// rt_mpc_qp/src/QP/QPBaseClass.h:49-51, QPBaseClass.cpp:111-112), batched.
//
// Replaces QPsolver_EiQuadProg::solve -> Eigen::QP::solve_quadprog
// (QPBaseClass.cpp:36-58, EiQuadProg.cpp:172-513) for the QPs the 16-lane
// kernel of qloco_gi.hip does not take (n > 16, p > 16 or m > 64); the C ABI
// (qloco_eiquadprog_solve) dispatches on size.  Same control flow (the l1 /
// l2 / l2a goto machine) and the same index quirks (SURVEY.md §8a-a20:
// me = p counts skipped zero CE columns, equality markers stored at A(i),
// the l1 / t1 loops start at me, delete_constraint searches from p; the
// uninitialised-index path reports QLOCO_UB_PATH) as qloco_gi_core.hpp.
//
// Mapping: one instance per 64-lane wavefront (one wave per workgroup), so
// every LDS hand-over is ordered by the wave itself (no barriers).  J and R
// (n x n, column-major, leading dimension n|1 -- odd, so a lane-per-row or a
// lane-per-column sweep is bank-conflict free for doubles) and the vectors
// live in dynamic LDS sized from (n, p, m): n = 60, m = 300 takes ~70 KB,
// two instances per CU.  Lane k owns row k (or column k) in the O(n^2)
// steps; the triangular solves are column sweeps (one v_readlane of the
// solved entry, then every lower lane updates its own accumulator) instead
// of the restatement's row-ordered sums, so results agree with the
// restatement to rounding, not bit for bit (tests/test_qp_gpu.py: status and
// iterations equal, x within 1e-9 relative); the dot products the active-set
// DECISIONS read (s, the step lengths, psi) keep the restatement's order.
// fp64, compiled without FMA contraction.
#include <float.h>
#include <math.h>
#include <string.h>
#include <mutex>

#include "qloco_common.hpp"
#include "qloco_gi_wide.hpp"

namespace qloco {

#define GW_SYNC() asm volatile("" ::: "memory")

__device__ __forceinline__ double gw_distance(double a, double b) {  // EiQuadProg.hpp:100-118
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

__device__ __forceinline__ double rl_d(double v, int l) {  // wave-uniform lane l
  const int64_t b = __builtin_bit_cast(int64_t, v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((int64_t)hi << 32) | (uint32_t)lo);
}

struct GwArgs {
  int n, p, m;
  int64_t batch;
  const double *G, *g0, *CE, *ce0, *CI, *ci0;
  int64_t sG, sg0, sCE, sce0, sCI, sci0;
  double *x, *f;
  int *status, *iters;
};

// dynamic LDS of one instance
struct GwLds {
  int n, ld, AS;
  double *J, *R, *x, *z, *d, *np, *xold, *s, *r, *u, *uold;
  int *A, *Aold, *iai, *iaexcl;
};

__host__ __device__ inline int gw_ld(int n) { return n | 1; }
__host__ __device__ inline int gw_as(int n, int p) { return (n > p ? n : p) + 1; }
__host__ __device__ inline size_t gw_lds_bytes(int n, int p, int m) {
  const int ld = gw_ld(n), as = gw_as(n, p);
  return sizeof(double) * (2 * (size_t)n * ld + 5 * (size_t)n + m + 3 * (size_t)as) +
         sizeof(int) * (2 * (size_t)as + 2 * (size_t)m);
}

__device__ __forceinline__ GwLds gw_carve(double *base, int n, int p, int m) {
  GwLds L;
  L.n = n;
  L.ld = gw_ld(n);
  L.AS = gw_as(n, p);
  double *q = base;
  L.J = q; q += (size_t)n * L.ld;
  L.R = q; q += (size_t)n * L.ld;
  L.x = q; q += n;
  L.z = q; q += n;
  L.d = q; q += n;
  L.np = q; q += n;
  L.xold = q; q += n;
  L.s = q; q += m;
  L.r = q; q += L.AS;
  L.u = q; q += L.AS;
  L.uold = q; q += L.AS;
  int *iq = reinterpret_cast<int *>(q);
  L.A = iq; iq += L.AS;
  L.Aold = iq; iq += L.AS;
  L.iai = iq; iq += m;
  L.iaexcl = iq;
  return L;
}

struct GwGroup {
  GwLds L;
  int li, n, p, m;
  const double *CE, *ce0, *CI, *ci0;
  __device__ __forceinline__ double &Jr(int r, int c) { return L.J[c * L.ld + r]; }
  __device__ __forceinline__ double &Rr(int r, int c) { return L.R[c * L.ld + r]; }
  __device__ __forceinline__ double CEc(int r, int i) const { return CE[(int64_t)i * n + r]; }
  __device__ __forceinline__ double CIc(int r, int i) const { return CI[(int64_t)i * n + r]; }

  // d = J' np : lane c sums its column in row order (EiQuadProg.hpp:121-124)
  __device__ __forceinline__ void compute_d() {
    const int c = li;
    if (c < n) {
      double acc = 0.0;
      for (int r = 0; r < n; ++r) acc += Jr(r, c) * L.np[r];
      L.d[c] = acc;
    }
    GW_SYNC();
  }
  // z = J(:, iq:) d(iq:) : lane r sums its row in column order (:126-129)
  __device__ __forceinline__ void update_z(int iq) {
    const int r = li;
    if (r < n) {
      double acc = 0.0;
      for (int c = iq; c < n; ++c) acc += Jr(r, c) * L.d[c];
      L.z[r] = acc;
    }
    GW_SYNC();
  }
  // r(0:iq) = triu(R)^-1 d(0:iq) (:131-134) as a column sweep: lane k holds
  // its right-hand side, the solved entry is read off its lane
  __device__ __forceinline__ void update_r(int iq) {
    double acc = li < iq ? L.d[li] : 0.0;
    double rk = 0.0;
    for (int i = iq - 1; i >= 0; --i) {
      const double ri = rl_d(acc, i) / L.R[i * L.ld + i];
      if (li == i) rk = ri;
      if (li < i) acc -= L.R[i * L.ld + li] * ri;
    }
    GW_SYNC();
    if (li < iq) L.r[li] = rk;
    GW_SYNC();
  }
  // EiQuadProg.cpp:30-93 ; false when degenerate.  The Givens parameters
  // come from d (every lane the same chain, the rotated entry carried in a
  // register), lane k rotates row k of J (its column j entry carried too).
  __device__ bool add_constraint(int &iq, double &R_norm) {
    const int k = li;
    if (n - 1 >= iq + 1) {
      double dcur = L.d[n - 1];
      double jcur = k < n ? Jr(k, n - 1) : 0.0;
      for (int j = n - 1; j >= iq + 1; j--) {
        double cc = L.d[j - 1];
        double ss = dcur;
        const double t1 = k < n ? Jr(k, j - 1) : 0.0;
        const double h = gw_distance(cc, ss);
        if (h == 0.0) {  // no rotation: column j keeps its current values
          if (k < n) Jr(k, j) = jcur;
          if (k == 0) L.d[j] = dcur;
          dcur = cc;
          jcur = t1;
          continue;
        }
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
        if (k == 0) L.d[j] = 0.0;
        const double xny = ss / (1.0 + cc);
        const double t2 = jcur;
        const double nj1 = t1 * cc + t2 * ss;
        if (k < n) Jr(k, j) = xny * (t1 + nj1) - t2;
        dcur = dj1;
        jcur = nj1;
      }
      if (k == 0) L.d[iq] = dcur;
      if (k < n) Jr(k, iq) = jcur;
    }
    GW_SYNC();
    iq++;
    if (li < iq) Rr(li, iq - 1) = L.d[li];
    GW_SYNC();
    const double dl = fabs(L.d[iq - 1]);
    if (dl <= DBL_EPSILON * R_norm) return false;
    if (dl > R_norm) R_norm = dl;
    return true;
  }
  // EiQuadProg.cpp:95-170 ; false on the reference's UB path
  __device__ bool delete_constraint(int p_, int &iq, int l) {
    int qq = -1;
    for (int i = p_; i < iq; i++)
      if (L.A[i] == l) {
        qq = i;
        break;
      }
    if (qq < 0) return false;
    // shift A / u / the R columns qq+1..iq-1 one place left (ascending,
    // in place: each column is read before it is overwritten)
    for (int i = qq; i < iq - 1; i++) {
      if (li < n) Rr(li, i) = L.R[(i + 1) * L.ld + li];
      if (li == 0) {
        L.A[i] = L.A[i + 1];
        L.u[i] = L.u[i + 1];
      }
      GW_SYNC();
    }
    if (li == 0) {
      L.A[iq - 1] = L.A[iq];
      L.u[iq - 1] = L.u[iq];
      L.A[iq] = 0;
      L.u[iq] = 0.0;
    }
    if (li < iq) Rr(li, iq - 1) = 0.0;
    GW_SYNC();
    iq--;
    if (iq == 0) return true;
    for (int j = qq; j < iq; j++) {
      double cc = L.R[j * L.ld + j];
      double ss = L.R[j * L.ld + j + 1];
      const double h = gw_distance(cc, ss);
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
      GW_SYNC();
      if (li == 0) {
        Rr(j + 1, j) = 0.0;
        Rr(j, j) = rjj;
      }
      {  // rows j, j+1 of R over columns k = j+1 .. iq-1 : lane k
        const int k = li;
        if (k >= j + 1 && k < iq) {
          const double t1 = L.R[k * L.ld + j];
          const double t2 = L.R[k * L.ld + j + 1];
          const double nj = t1 * cc + t2 * ss;
          Rr(j, k) = nj;
          Rr(j + 1, k) = xny * (t1 + nj) - t2;
        }
      }
      {  // columns j, j+1 of J : lane = row
        const int k = li;
        if (k < n) {
          const double t1 = Jr(k, j);
          const double t2 = Jr(k, j + 1);
          const double nj = t1 * cc + t2 * ss;
          Jr(k, j) = nj;
          Jr(k, j + 1) = xny * (nj + t1) - t2;
        }
      }
      GW_SYNC();
    }
    return true;
  }
};

__device__ void gw_solve(GwLds L, int li, int n, int p, int m, const double *G, const double *g0,
                         const double *CE, const double *ce0, const double *CI,
                         const double *ci0, double *xout, double &f_out, int &status_out,
                         int &iters_out) {
  GwGroup g;
  g.L = L;
  g.li = li;
  g.n = n;
  g.p = p;
  g.m = m;
  g.CE = CE;
  g.ce0 = ce0;
  g.CI = CI;
  g.ci0 = ci0;
  const int ld = L.ld;
  const double inf = INFINITY;
  int status = QLOCO_OK;
  int iter = 0;
  double f_value = 0.0;
  for (int k = li; k < L.AS; k += 64) {
    L.A[k] = 0;
    L.Aold[k] = 0;
    L.u[k] = 0.0;
    L.r[k] = 0.0;
    L.uold[k] = 0.0;
  }
  for (int k = li; k < m; k += 64) {
    L.iai[k] = 0;
    L.iaexcl[k] = 0;
  }
  // ---- solve_quadprog: c1 = trace(G); LLT of the lower triangle (EiQuadProg.cpp:493-513)
  double c1 = 0.0;
  for (int i = 0; i < n; ++i) c1 += G[(int64_t)i * n + i];
  if (li < n)
    for (int c = 0; c < n; ++c) L.R[c * ld + li] = c <= li ? G[(int64_t)c * n + li] : 0.0;
  GW_SYNC();
  bool pd = true;
  for (int k = 0; k < n; ++k) {
    double x = L.R[k * ld + k];
    for (int j = 0; j < k; ++j) x -= L.R[j * ld + k] * L.R[j * ld + k];
    if (!(x > 0.0)) {
      pd = false;
      break;
    }
    const double lkk = sqrt(x);
    const int r = li;
    double lrk = 0.0;
    if (r > k && r < n) {
      double acc = L.R[k * ld + r];
      for (int j = 0; j < k; ++j) acc -= L.R[j * ld + r] * L.R[j * ld + k];
      lrk = acc / lkk;
    }
    GW_SYNC();
    if (r > k && r < n) L.R[k * ld + r] = lrk;
    if (li == 0) L.R[k * ld + k] = lkk;
    GW_SYNC();
  }
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
        for (int j = rr + 1; j < n; ++j) acc -= L.R[rr * ld + j] * L.J[c * ld + j];
        L.J[c * ld + rr] = acc / L.R[rr * ld + rr];
      }
    }
    GW_SYNC();
    double c2 = 0.0;
    for (int i = 0; i < n; ++i) c2 += L.J[i * ld + i];
    // x = -G^-1 g0 through the factor (:227-230), column sweeps
    {
      double acc = li < n ? g0[li] : 0.0, xi = 0.0;
      for (int i = 0; i < n; ++i) {  // L y = g0
        const double yi = rl_d(acc, i) / L.R[i * ld + i];
        if (li == i) xi = yi;
        if (li > i && li < n) acc -= L.R[i * ld + li] * yi;
      }
      acc = xi;
      for (int i = n - 1; i >= 0; --i) {  // L' x = y
        const double v = rl_d(acc, i) / L.R[i * ld + i];
        if (li == i) xi = v;
        if (li < i) acc -= L.R[li * ld + i] * v;
      }
      GW_SYNC();
      if (li < n) L.x[li] = -xi;
    }
    GW_SYNC();
    f_value = 0.0;
    for (int i = 0; i < n; ++i) f_value += g0[i] * L.x[i];
    f_value *= 0.5;
    // solve_quadprog2 preprocessing: d = 0, R = 0, R_norm = 1 (:207-209)
    for (int c = 0; c < n; ++c)
      if (li < n) L.R[c * ld + li] = 0.0;
    if (li < n) L.d[li] = 0.0;
    GW_SYNC();
    double R_norm = 1.0;
    const int me = p, mi = m;
    int iq = 0;
    int ip = 0, l = 0;
    double ss = 0.0, psi, t, t1, t2;

    // ---- equality constraints (:237-276), quirks kept; all-zero CE
    // columns are skipped (:239-244)
    for (int i = 0; i < me; i++) {
      const bool nzl = li < n && g.CEc(li, i) != 0.0;
      if (!__ballot(nzl)) continue;
      if (li < n) L.np[li] = g.CEc(li, i);
      GW_SYNC();
      g.compute_d();
      g.update_z(iq);
      g.update_r(iq);
      t2 = 0.0;
      double zz = 0.0, znp = 0.0, npx = 0.0;
      for (int k = 0; k < n; ++k) {
        zz += L.z[k] * L.z[k];
        znp += L.z[k] * L.np[k];
        npx += L.np[k] * L.x[k];
      }
      if (fabs(zz) > DBL_EPSILON) t2 = (-npx - g.ce0[i]) / znp;
      GW_SYNC();
      if (li < n) L.x[li] += t2 * L.z[li];
      for (int k = li; k < iq; k += 64) L.u[k] -= t2 * L.r[k];
      if (li == 0) {
        L.u[iq] = t2;
        L.A[i] = -i - 1;
      }
      GW_SYNC();
      f_value += 0.5 * (t2 * t2) * znp;
      if (!g.add_constraint(iq, R_norm)) {
        status = QLOCO_DEGENERATE;
        goto done;
      }
    }
    for (int i = li; i < mi; i += 64) L.iai[i] = i;
    GW_SYNC();

  l1:
    iter++;
    GW_SYNC();
    for (int i = me + li; i < iq; i += 64) L.iai[L.A[i]] = -1;
    GW_SYNC();
    ss = 0.0;
    psi = 0.0;
    ip = 0;
    // s(x) = CI' x + ci0, one constraint per lane, row order
    for (int i = li; i < mi; i += 64) {
      L.iaexcl[i] = 1;
      double sum = 0.0;
      for (int r = 0; r < n; ++r) sum += g.CIc(r, i) * L.x[r];
      L.s[i] = sum + g.ci0[i];
    }
    GW_SYNC();
    for (int i = 0; i < mi; i++) psi += (L.s[i] < 0.0) ? L.s[i] : 0.0;
    if (fabs(psi) <= mi * DBL_EPSILON * c1 * c2 * 100.0) goto done;
    GW_SYNC();
    for (int i = li; i < iq; i += 64) {
      L.uold[i] = L.u[i];
      L.Aold[i] = L.A[i];
    }
    if (li < n) L.xold[li] = L.x[li];
    GW_SYNC();

  l2:
    {
      // the first strict minimum below ss over the admissible constraints
      // (the restatement's ascending scan, ss kept across goto l2): lane
      // minima, then (value, index) pairs reduced across the wave
      double bv = ss;
      int bi = -1;
      for (int i = li; i < mi; i += 64)
        if (L.s[i] < bv && L.iai[i] != -1 && L.iaexcl[i]) {
          bv = L.s[i];
          bi = i;
        }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (oi >= 0 && (bi < 0 || ov < bv || (ov == bv && oi < bi))) {
          bv = ov;
          bi = oi;
        }
      }
      bi = __builtin_amdgcn_readfirstlane(bi);
      if (bi >= 0) {
        ss = rl_d(bv, 0);
        ip = bi;
      }
    }
    if (ss >= 0.0) goto done;
    GW_SYNC();
    if (li < n) L.np[li] = g.CIc(li, ip);
    if (li == 0) {
      L.u[iq] = 0.0;
      L.A[iq] = ip;
    }
    GW_SYNC();

  l2a:
    g.compute_d();
    g.update_z(iq);
    g.update_r(iq);
    l = 0;
    t1 = inf;
    for (int k = me; k < iq; k++) {
      double tmp;
      if (L.r[k] > 0.0 && ((tmp = L.u[k] / L.r[k]) < t1)) {
        t1 = tmp;
        l = L.A[k];
      }
    }
    {
      double zz = 0.0, znp = 0.0;
      for (int k = 0; k < n; ++k) {
        zz += L.z[k] * L.z[k];
        znp += L.z[k] * L.np[k];
      }
      if (fabs(zz) > DBL_EPSILON)
        t2 = -L.s[ip] / znp;
      else
        t2 = inf;
      t = (t1 < t2) ? t1 : t2;
      if (t >= inf) {
        status = QLOCO_INFEASIBLE;
        f_value = inf;
        goto done;
      }
      if (t2 >= inf) {
        GW_SYNC();
        for (int k = li; k < iq; k += 64) L.u[k] -= t * L.r[k];
        if (li == 0) {
          L.u[iq] += t;
          L.iai[l] = l;
        }
        GW_SYNC();
        if (!g.delete_constraint(p, iq, l)) {
          status = QLOCO_UB_PATH;
          goto done;
        }
        goto l2a;
      }
      GW_SYNC();
      if (li < n) L.x[li] += t * L.z[li];
      f_value += t * znp * (0.5 * t + L.u[iq]);
      GW_SYNC();
      for (int k = li; k < iq; k += 64) L.u[k] -= t * L.r[k];
      if (li == 0) L.u[iq] += t;
      GW_SYNC();
    }
    if (t == t2) {
      if (!g.add_constraint(iq, R_norm)) {
        GW_SYNC();
        if (li == 0) L.iaexcl[ip] = 0;
        GW_SYNC();
        if (!g.delete_constraint(p, iq, ip)) {
          status = QLOCO_UB_PATH;
          goto done;
        }
        for (int i = li; i < m; i += 64) L.iai[i] = i;
        GW_SYNC();
        bool bad = false;
        for (int i = 0; i < iq; i++) bad = bad || (L.Aold[i] < 0 || L.Aold[i] >= m);
        if (bad) {  // reference: out-of-range write through _iai(_A(i)), UB
          status = QLOCO_UB_PATH;
          goto done;
        }
        if (li == 0)
          for (int i = 0; i < iq; i++) {
            L.A[i] = L.Aold[i];
            L.iai[L.A[i]] = -1;
            L.u[i] = L.uold[i];
          }
        if (li < n) L.x[li] = L.xold[li];
        GW_SYNC();
        goto l2;
      } else {
        GW_SYNC();
        if (li == 0) L.iai[ip] = -1;
        GW_SYNC();
      }
      goto l1;
    }
    // partial step: drop constraint l (:477-490)
    GW_SYNC();
    if (li == 0) L.iai[l] = l;
    GW_SYNC();
    if (!g.delete_constraint(p, iq, l)) {
      status = QLOCO_UB_PATH;
      goto done;
    }
    {
      double sum = 0.0;
      for (int r = 0; r < n; ++r) sum += g.CIc(r, ip) * L.x[r];
      GW_SYNC();
      if (li == 0) L.s[ip] = sum + g.ci0[ip];
      GW_SYNC();
    }
    goto l2a;
  }

done:
  GW_SYNC();
  if (li < n) xout[li] = L.x[li];
  f_out = f_value;
  status_out = status;
  iters_out = iter;
  GW_SYNC();
}

__global__ __launch_bounds__(64) void gi_wide_kernel(const GwArgs a) {
  extern __shared__ double gw_smem[];
  const int64_t inst = blockIdx.x;
  if (inst >= a.batch) return;
  const int li = threadIdx.x;
  GwLds L = gw_carve(gw_smem, a.n, a.p, a.m);
  double f;
  int st, it;
  gw_solve(L, li, a.n, a.p, a.m, a.G + inst * a.sG, a.g0 + inst * a.sg0,
           a.CE ? a.CE + inst * a.sCE : nullptr, a.ce0 ? a.ce0 + inst * a.sce0 : nullptr,
           a.CI ? a.CI + inst * a.sCI : nullptr, a.ci0 ? a.ci0 + inst * a.sci0 : nullptr,
           a.x + inst * a.n, f, st, it);
  if (li == 0) {
    if (a.f) a.f[inst] = f;
    if (a.status) a.status[inst] = st;
    if (a.iters) a.iters[inst] = it;
  }
}

int gi_wide_launch(int n, int p, int m, int64_t batch, const double *G, int64_t sG,
                   const double *g0, int64_t sg0, const double *CE, int64_t sCE,
                   const double *ce0, int64_t sce0, const double *CI, int64_t sCI,
                   const double *ci0, int64_t sci0, double *x, double *f, int32_t *status,
                   int32_t *iters, hipStream_t stream) {
  if (n < 1 || n > kGiWideN || p < 0 || p > kGiWideP || m < 0 || m > kGiWideM)
    return QLOCO_BAD_SIZE;
  GwArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.p = p;
  a.m = m;
  a.batch = batch;
  a.G = G;
  a.g0 = g0;
  a.CE = CE;
  a.ce0 = ce0;
  a.CI = CI;
  a.ci0 = ci0;
  a.sG = sG;
  a.sg0 = sg0;
  a.sCE = sCE;
  a.sce0 = sce0;
  a.sCI = sCI;
  a.sci0 = sci0;
  a.x = x;
  a.f = f;
  a.status = status;
  a.iters = iters;
  const size_t lds = gw_lds_bytes(n, p, m);
  // dynamic LDS beyond the 64 KB default needs the attribute, set once per
  // device; a device that refuses it cannot run the larger shapes, and the
  // caller is told why instead of getting a generic launch failure
  if (lds > 64 * 1024) {
    static std::mutex mu;
    static int state[64] = {0};  // per device: 0 unknown, 1 set, -1 refused
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return QLOCO_ERR_DEVICE;
    std::lock_guard<std::mutex> lk(mu);
    if (state[dev] == 0) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(gi_wide_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      state[dev] = e == hipSuccess ? 1 : -1;
      if (e != hipSuccess) {
        set_last_error("gi_wide_kernel: the device refused 160 KB of dynamic LDS "
                       "(hipFuncAttributeMaxDynamicSharedMemorySize); shapes needing more than "
                       "64 KB cannot run",
                       e);
        (void)hipGetLastError();
      }
    }
    if (state[dev] < 0) return QLOCO_BAD_SIZE;
  }
  hipLaunchKernelGGL(gi_wide_kernel, dim3((unsigned)batch), dim3(64), lds, stream, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "gi_wide_kernel launch");
  return QLOCO_OK;
}

}  // namespace qloco
