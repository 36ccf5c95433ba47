// qloco_srbd.hip -- batched SRBD convex MPC for gfx950 (MI355X).
//
// Replaces the reference's per-call ConvexMpc build + OSQP solve
// (a1_cpp_open_source/src/ConvexMpc.cpp:8-264, A1RobotControl.cpp:452-600)
// with ONE fused kernel: one QP instance per workgroup of W wavefronts
// (W = 1 for <= 63 stance variables, W = 2 for <= 126), nothing but the
// inputs and the solution touching HBM.
//
// Design (DESIGN.md §3 has the derivation):
//  * Swing legs are eliminated exactly: their bounds fz in [0, 0] with the
//    friction rows force f = 0, so only stance forces are variables
//    (n = 3 * #stance (step, leg) pairs, 5 constraint rows per stance leg).
//  * The condensed Hessian H = Bqp' Q Bqp + R is generated in closed form.
//    With forward Euler and the reference's A_c (ConvexMpc.cpp:111-133),
//    A_c is nilpotent, so A_d^k B_d = B_d + k dt A_c B_d and every B_qp
//    block is b + (i-j) e with b (rows 6..11) and e (rows 0..5) disjoint:
//    H[r][c] = K0(j_r,j_c) * <b_r,b_c>_Q + K2(j_r,j_c) * <e_r,e_c>_Q + R,
//    K0 = #{i >= max(j_r,j_c)}, K2 = sum_i (i-j_r)(i-j_c).  Bqp x and
//    Bqp' w (gradient, P x for the residuals) are per-step prefix / suffix
//    sums computed by all lanes in parallel.
//  * ADMM is OSQP's algorithm (Ruiz scaling, rho vector, relaxation,
//    termination every check_termination iterations, adaptive rho) in fp32.
//    Lane v owns stance variable v (leg triples never straddle a wave:
//    21 legs = 63 lanes per wave, lane 63 pads), its row of K^-1 in up to
//    64*W VGPRs (K = P + sigma I + A' diag(rho) A, inverted in
//    place by Gauss-Jordan), and the <= 2 constraint rows of its leg's 5
//    (x: rows 0,1; y: rows 2,3; z: row 4).  Padding lanes carry zero A rows,
//    zero q and so a zero right-hand side; their K rows are the identity row
//    where the diagonal falls inside the columns a form keeps (NK), a zero
//    row past it (the narrowed forms allocate no padding columns), and either
//    way their x_tilde is 0 -- every loop over columns is straight-line code.
//    Per iteration: one LDS broadcast of the KKT right-hand side, one matvec
//    against the register-resident K^-1 (one v_fmac_f32_dpp row_newbcast per
//    entry, qloco_dpp.inc), DPP lane shifts (wave_shr/wave_shl) for the
//    leg-local constraint couplings.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include <type_traits>

#include "qloco_common.hpp"
#include "qloco_srbd_core.hpp"

// The KKT inverse is the register-row DPP Gauss-Jordan below.  The
// matrix-core block Gauss-Jordan forms measured against it (as accurate once
// made stable, but slower) live in
// tools/micro/srbd_mfma_inverse.inc with their probe.

namespace qloco {

constexpr int kMaxN = 20;    // max horizon compiled in (BASELINE configs: N <= 20)
constexpr int kLegsPerWave = 21;
// The one-wave class takes instances of at most kW1Legs stance legs.  20
// (60 variables, every Go1 trot / pace N = 10 instance) lets the one-wave
// kernel carry a single 60-column form of its inverse, matvec and Ruiz
// sweeps -- 124 -> ~80 KB of code; 21-leg instances then go to the two-wave
// class.  21 keeps the 64-column forms as well.
constexpr int kW1Legs = 20;
static_assert(kW1Legs == 20 || kW1Legs == 21, "one-wave class: 20 or 21 legs");



// NM: the largest horizon the instantiation admits (per-step tables are
// sized by it: NM = 10 keeps the one-wave workgroup under 10 KB of LDS, so
// 16 fit a CU -- four waves per SIMD)
template <int W, int NM = kMaxN>
struct SrbdLds {
  static constexpr int NC = 64 * W;
  f4v bc[2][NC / 4];       // broadcast ring (KKT rhs, GJ pivot rows, Ruiz D)
  f4v bv[NC][2];           // per var: {b0,b1,b2,e0}, {e1,e2,step,comp}
  float xs[NC];            // unscaled x per var (P x)
  float Dc[NC];            // Ruiz column scaling D
  float err[12 * NM];   // per-step row values (gradient error / aggregates)
  float Wc[12 * NM];    // per-step Bqp' weights: rows 0..5 W1, rows 6..11 W0
  float q2[16];
  float r2[12];
  float x0[16];
  float aux[3][NC];         // per var, read off the hot path: 2 r (R diag), E row0, E row1
  f4v zb[NC];               // per var: scaled bounds (l0, u0, l1, u1) of its 2 slots
  f4v arz[NC];              // per var: scaled A entries (ra0, ra1, rz0, rz1) of its 2 slots
  float qs[NC];             // per var: scaled q
  int pair[NC];             // per var: 4*step + leg
  int cst[NC];              // per var: step, NM on padding (row of zeros in k0k2)
  f2v k0k2[NM * (NM + 1)];  // [row step][col step]: horizon sums K0, K2
  float piv[2];
  float qn[2];              // ||D^-1 q||_inf, ||q||_inf (scaled): read at the checks
  float colv[W == 1 ? 1 : 2][W == 1 ? 1 : NC];  // W = 2 inverse: pivot column
  float red[W][16];
  int legtab[4 * NM];   // stance pair -> 4*step + leg
  int stepstart[NM + 1];
  int nlegs;
  uint8_t ct[4 * NM];
};

// LDS ordering between the lanes of ONE wave needs no s_barrier (a wave's
// LDS instructions execute in order); only the compiler must not move
// memory operations across the point.
template <int W>
__device__ __forceinline__ void bsync() {
  if constexpr (W == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}


// Block-wide max of NON-NEGATIVE values (residual norms, |q|).
template <int W, int NV>
__device__ __forceinline__ void bmax(float (&v)[NV], float (*red)[16]) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wmax_nonneg(v[k]);
  if constexpr (W > 1) {
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < NV; ++k) red[wave][k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float r = red[0][k];
#pragma unroll
      for (int w = 1; w < W; ++w) r = fmaxf(r, red[w][k]);
      v[k] = uni(r);
    }
    __syncthreads();
  }
}
template <int W>
__device__ __forceinline__ float bsum(float v, float (*red)[16]) {
  v = wsum(v);
  if constexpr (W > 1) {
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[wave][15] = v;
    __syncthreads();
    float r = red[0][15];
#pragma unroll
    for (int w = 1; w < W; ++w) r += red[w][15];
    v = uni(r);
    __syncthreads();
  }
  return v;
}

// (Bqp' w)_v for a variable of step `step`, component `comp`, from S.Wc.
template <int W, int NM>
__device__ __forceinline__ float bqp_t(const SrbdLds<W, NM> &S, int step, int comp, f4v lo, f4v hi,
                                       float dtm, float dt2m) {
  const float *w = S.Wc + 12 * step;
  float acc = lo.x * w[6] + lo.y * w[7] + lo.z * w[8];
  acc += lo.w * w[0] + hi.x * w[1] + hi.y * w[2];
  acc += dtm * w[9 + comp] + dt2m * w[3 + comp];
  return acc;
}

// Per-row scans over the horizon, lanes r < 12 (one row each), the N
// values read up front (unconditional in-bounds loads, one wait), the
// recurrences in registers behind uniform step guards.
//  forward (P x only): S.err[i][r] <- q2[r] * s_i[r], s_i = sum_{j<=i} agg_j
//      on b rows (6..11), sum_{j<i} (i-j) agg_j on e rows (0..5);
//  suffix: S.Wc[j][r] = sum_{i>=j} wt(i-j) S.err[i][r]; wt = 1 on b rows
//      (W0), (i-j) on e rows (W1).
template <int W, int NM>
__device__ __forceinline__ void row_scans(SrbdLds<W, NM> &S, int N, bool forward) {
  const int r = opaque_tid();
  if (r >= 12) return;
  const bool brow = r >= 6;
  float v[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) v[i] = S.err[12 * i + r];
  if (forward) {
    const float q = S.q2[r];
    float pa = 0.0f, pe = 0.0f, se = 0.0f;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      if (i < N) {
        se += pe;
        pe += v[i];
        pa += v[i];
        v[i] = q * (brow ? pa : se);
      }
    }
  }
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int j = NM - 1; j >= 0; --j) {
    if (j < N) {
      s1 += s0;  // S1[j] = S1[j+1] + S0[j+1]
      s0 += v[j];
      S.Wc[12 * j + r] = brow ? s0 : s1;
    }
  }
}

// P x phase (b) in one pass: the prefix scan over steps, Q and the weighted
// suffix scan compose to W[j][r] = q2[r] sum_k Kx(j,k) agg_k[r] with Kx = K0
// on b rows and K2 on e rows -- the horizon sums of the k0k2 table
// (sum_{i >= max(j,k)} 1 and sum_{i >= max(j,k)} (i-j)(i-k)).  All lanes, 12N
// outputs, the table row and the aggregates read up front when NB (= N) is
// a compile-time constant (N = 10); other horizons use rolled loops.
template <int W, int NB, int NM>
__device__ __forceinline__ void horizon_rows(SrbdLds<W, NM> &S, int N) {
  constexpr int NT = 64 * W;
  if constexpr (NB == 0) {  // any horizon: rolled loops (cold configurations)
    for (int idx = opaque_tid(); idx < 12 * N; idx += NT) {
      const int j = idx / 12, r = idx - 12 * j;
      const f2v *kr = &S.k0k2[j * (NM + 1)];
      float acc = 0.0f;
      for (int k = 0; k < N; ++k) acc = fmaf(r >= 6 ? kr[k].x : kr[k].y, S.err[12 * k + r], acc);
      S.Wc[idx] = S.q2[r] * acc;
    }
    return;
  }
#pragma unroll
  for (int pass = 0; pass < (12 * (NB > 0 ? NB : 1) + NT - 1) / NT; ++pass) {
    const int idx = opaque_tid() + NT * pass;
    if (idx < 12 * N) {
      const int j = idx / 12, r = idx - 12 * j;
      const f2v *kr = &S.k0k2[j * (NM + 1)];
      float a0 = 0.0f, a1 = 0.0f;
      if (r >= 6) {
#pragma unroll
        for (int k = 0; k < NB; k += 2) {
          a0 = fmaf(kr[k].x, S.err[12 * k + r], a0);
          if (k + 1 < NB) a1 = fmaf(kr[k + 1].x, S.err[12 * (k + 1) + r], a1);
        }
      } else {
#pragma unroll
        for (int k = 0; k < NB; k += 2) {
          a0 = fmaf(kr[k].y, S.err[12 * k + r], a0);
          if (k + 1 < NB) a1 = fmaf(kr[k + 1].y, S.err[12 * (k + 1) + r], a1);
        }
      }
      S.Wc[idx] = S.q2[r] * (a0 + a1);
    }
  }
}

// Unscaled (P x)_v, P = Bqp' Q Bqp + R.  Caller has written S.xs (unscaled
// x, 0 on padding) and synced.  Three phases, all lanes busy:
//  (a) per-step aggregates agg_j[s] = sum_{v in step j} Bcoef(v, s) x_v
//  (b) state rows s_i (b rows: prefix sum, e rows: weighted prefix sum),
//      w_i = Q s_i, suffix weights W0 / W1 per (j, r) -> S.Wc (horizon_rows)
//  (c) this lane's (Bqp' w)_v + R x_v
template <int W, int NM>
__device__ __forceinline__ float p_times_x(SrbdLds<W, NM> &S, int N, bool valid, int step, int comp,
                                           f4v lo, f4v hi, float r2v, float xu, float dtm,
                                           float dt2m) {
  const int t = opaque_tid();
  for (int idx = t; idx < 12 * N; idx += 64 * W) {
    const int j = idx / 12, s = idx - 12 * j;
    const int sg = s / 3, sc = s - 3 * sg;  // 0: e rows, 1: p rows, 2: b rows, 3: v rows
    const int off = (sg == 0 ? 3 : 0) + sc;
    const float dsc = sg == 1 ? dt2m : dtm;
    const int p0 = S.stepstart[j], p1 = S.stepstart[j + 1];
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // loads from a valid pair on every lane (pair 0 when past the step's
      // last), the term masked: the 24 LDS reads issue together instead of
      // one divergent round trip per pair
      const int p = p0 + q;
      const bool ok = p < p1;
      const int pc = ok ? p : 0;
      const int vb = 64 * (pc / kLegsPerWave) + 3 * (pc % kLegsPerWave);
      const float *bf = reinterpret_cast<const float *>(&S.bv[vb][0]);
      const float xa = S.xs[vb], xb = S.xs[vb + 1], xc = S.xs[vb + 2];
      const float ev = bf[off] * xa + bf[8 + off] * xb + bf[16 + off] * xc;
      const float xsel = sc == 0 ? xa : (sc == 1 ? xb : xc);
      const float term = (sg & 1) ? dsc * xsel : ev;
      acc += ok ? term : 0.0f;
    }
    S.err[idx] = acc;
  }
  bsync<W>();
  if (N == 10) {
    horizon_rows<W, 10>(S, N);
  } else {
    horizon_rows<W, 0>(S, N);
  }
  bsync<W>();
  return valid ? bqp_t<W>(S, step, comp, lo, hi, dtm, dt2m) + r2v * xu : 0.0f;
}


// This lane's coefficients for the closed-form P row.
struct PCoef {
  float bq0, bq1, bq2, eq0, eq1, eq2, linb, line;
};
template <int W, int NM>
__device__ __forceinline__ PCoef p_coef(const SrbdLds<W, NM> &S, f4v lo, f4v hi, int comp, bool valid,
                                        float dtm, float dt2m) {
  PCoef c;
  c.bq0 = S.q2[6] * lo.x;
  c.bq1 = S.q2[7] * lo.y;
  c.bq2 = S.q2[8] * lo.z;
  c.eq0 = S.q2[0] * lo.w;
  c.eq1 = S.q2[1] * hi.x;
  c.eq2 = S.q2[2] * hi.y;
  c.linb = valid ? S.q2[9 + comp] * dtm * dtm : 0.0f;
  c.line = valid ? S.q2[3 + comp] * dt2m * dt2m : 0.0f;
  return c;
}

// Unscaled closed-form P row (padding rows: the identity row).  Columns
// come in leg triples (lanes 3l..3l+2 of a wave, lane 63 padding), so the
// column component is static and K0 / K2 -- functions of the row and column
// steps only -- are one LDS table read per triple.
template <int W, int C2, int NM>
__device__ __forceinline__ void gen_p_row(const SrbdLds<W, NM> &S, const PCoef &pc, int t, bool valid,
                                          int step, int comp, float r2v, Row<W> &K) {
  // opaque copies: keep LICM from hoisting per-column selects out of the ADMM loop
  int tt = t, kb = step * (NM + 1);
  // padding lanes have zero coefficients, so only their diagonal needs a 1
  float dadd = valid ? r2v : 1.0f;
  float lb0 = comp == 0 ? pc.linb : 0.0f, lb1 = comp == 1 ? pc.linb : 0.0f,
        lb2 = comp == 2 ? pc.linb : 0.0f;
  float le0 = comp == 0 ? pc.line : 0.0f, le1 = comp == 1 ? pc.line : 0.0f,
        le2 = comp == 2 ? pc.line : 0.0f;
  asm volatile("" : "+v"(tt), "+v"(kb), "+v"(dadd), "+v"(lb0), "+v"(lb1), "+v"(lb2), "+v"(le0),
               "+v"(le1), "+v"(le2));
#pragma unroll
  for (int h = 0; h < W; ++h) {
    // the second half of a two-wave row stops at its bucket's 4 C2 columns,
    // a one-wave row at kW1Legs legs (60 columns: 60..63 never allocated)
    constexpr bool kNarrow = W == 2 && C2 < 16;
    constexpr bool kW1Narrow = W == 1 && kW1Legs <= 20;
#pragma unroll
    for (int l = 0; l < ((h == 1 && kNarrow) ? 4 * C2 / 3 : (kW1Narrow ? kW1Legs : kLegsPerWave)); ++l) {
      __builtin_amdgcn_sched_barrier(0);  // bound live ranges: one triple at a time
      const int c0 = 64 * h + 3 * l;
      const f2v kk = S.k0k2[kb + S.cst[c0]];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c = c0 + j;
        const f4v lo = S.bv[c][0], hi = S.bv[c][1];
        const float lb = j == 0 ? lb0 : (j == 1 ? lb1 : lb2);
        const float le = j == 0 ? le0 : (j == 1 ? le1 : le2);
        const float beta = fmaf(pc.bq2, lo.z, fmaf(pc.bq1, lo.y, fmaf(pc.bq0, lo.x, lb)));
        const float epsv = fmaf(pc.eq2, hi.y, fmaf(pc.eq1, hi.x, fmaf(pc.eq0, lo.w, le)));
        float pv = fmaf(kk.y, epsv, kk.x * beta);
        pv += (c == tt) ? dadd : 0.0f;
        KE(K, c) = pv;
      }
    }
    if (!(h == 1 && kNarrow) && !kW1Narrow)
      KE(K, 64 * h + 63) = (64 * h + 63 == tt) ? dadd : 0.0f;  // padding column
  }
}

// W = 2: the second half of a row (columns 64..) holds ncol[1] valid
// columns.  Each two-wave kernel is instantiated for one bucket C2 of them
// (3, 6, 9 or 15 DPP chunks: <= 12, 24, 36 or 60 columns, i.e. 21-25, 26-29,
// 30-33 or 34-41 stance legs; 42 legs go to the wide kernel); the padding
// columns beyond are identity (zero on valid rows), so the shorter forms
// are exact, and the registers of the columns a bucket never touches are
// not allocated at all.
constexpr int w2_bucket_legs(int c2) { return kLegsPerWave + (c2 < 16 ? 4 * c2 / 3 : kLegsPerWave); }
#define QL_HALF2(C2, NAME12, NAME24, NAME36, NAME60, NAME64, ...) \
  do {                                                           \
    if constexpr ((C2) == 3) {                                   \
      NAME12(__VA_ARGS__);                                       \
    } else if constexpr ((C2) == 6) {                            \
      NAME24(__VA_ARGS__);                                       \
    } else if constexpr ((C2) == 9) {                            \
      NAME36(__VA_ARGS__);                                       \
    } else if constexpr ((C2) == 15) {                           \
      NAME60(__VA_ARGS__);                                       \
    } else {                                                     \
      NAME64(__VA_ARGS__);                                       \
    }                                                            \
  } while (0)

// K_rc <- rs * D_c * P_rc + [sigma I + A' diag(rho) A]_rc, the leg block
// touching only the lane's own leg columns (static column -> leg map; D_c
// fanned out from one LDS chunk per lane by DPP).  Returns the diagonal
// (pivot tracking of the W = 2 inverse).
template <int W, int C2, int NM>
__device__ __forceinline__ float finalize_row(const SrbdLds<W, NM> &S, int t, int cbase, float rs,
                                              float add0, float add1, float add2, bool c60,
                                              Row<W> &K) {
  constexpr int NC = W == 1 ? (kW1Legs <= 20 ? 60 : 64) : 64 + 4 * C2;
  const int lane = t & 63;
  const f4v d0 = reinterpret_cast<const f4v *>(S.Dc)[lane & 15];
  if (W == 1 && c60) {  // padding columns 60..63 have D = 1
    QL_DPP_MUL60(K.k, 0, d0);
  } else {
    QL_DPP_MUL64(K.k, 0, d0);
  }
  if constexpr (W == 2) {
    const f4v d1 = reinterpret_cast<const f4v *>(S.Dc)[16 + (lane & 15)];
    QL_HALF2(C2, QL_DPP_MUL12, QL_DPP_MUL24, QL_DPP_MUL36, QL_DPP_MUL60, QL_DPP_MUL64, K.k, 64, d1);
  }
  int cb = cbase, tt = t;
  asm volatile("" : "+v"(cb), "+v"(tt));
  float diag = 1.0f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cl = c & 63, lb = (c & ~63) + 3 * (cl / 3);  // leg base column of c
    const int o = cl - 3 * (cl / 3);
    const bool own = (cb == lb);
    const float ad = own ? (o == 0 ? add0 : (o == 1 ? add1 : add2)) : 0.0f;
    const float v = fmaf(KE(K, c), rs, ad);
    KE(K, c) = v;
    if constexpr (W == 2) diag = (c == tt) ? v : diag;
  }
  return diag;
}

// In-place Gauss-Jordan inverse of the register-resident SPD K (no
// pivoting; Ruiz-scaled).  Step k: every row r takes
//   A_rc <- A_rc - g_r * (pivot row)_c,  g_r = A_rk / p   (one DPP FMA per column)
// with the pivot row's own scaling by 1/p folded into the same FMA
// (g_k = 1 - 1/p against the row plus the identity, e_k = p + 1).  That fused
// form rounds 1 - 1/p and carries a relative error ~p*eps into column k, so
// for a large pivot (p > kGjExactPivot) column k is then written exactly
// (A_kk = 1/p, A_rk = -g_r): the literal QP's equality rows (rho_eq = 1e3 rho)
// reach p ~ 3e5, where the fused column was 1e3x off and ADMM diverged
// (DESIGN.md §3e).  Small pivots keep the fused column, whose rounding is
// shared with the pivot row (measured the more accurate at eps 1e-6).  GJ on a
// symmetric matrix keeps A_kc = +A_ck for unprocessed c and -A_ck for
// processed c (< k), so every lane writes its own column-k entry as the pivot
// row (a static register: the pivot loop is unrolled) and the pivot is a
// v_readlane -- one coalesced ds_write_b32 and one ds_read_b128 per pivot,
// the row fanned out by DPP.  Only the valid pivots run; padding rows never
// change: identity rows inside the kept columns, zero rows past them (the
// narrowed forms stop at NK), both with a zero right-hand side.

template <bool C60, int NM>
__device__ __forceinline__ void invert_w1(SrbdLds<1, NM> &S, int t, int ncol, Row<1> &K) {
  const int lane = t & 63;
  int nc = __builtin_amdgcn_readfirstlane(ncol);
  // pivots emitted: 60 when the one-wave class stops at 20 legs (code size)
  constexpr int KP = (C60 && kW1Legs <= 20) ? 60 : 64;
  // one pivot of look-ahead: pivot k applies its update to column k + 1 first
  // (the same fused multiply-add the full update performs: bit-identical) and
  // publishes pivot k + 1's row, which is in flight during the other columns
  {
    const float v = K.k[0];
    const float p = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    reinterpret_cast<float *>(&S.bc[0][0])[lane] = lane == 0 ? p + 1.0f : v;
  }
  ColLoop<0, KP>::run([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    asm volatile("" : "+s"(nc));  // the per-pivot compare stays a scalar one (not 64 hoisted masks)
    if (k >= nc) return;  // wave-uniform (static register k: the pivot loop is unrolled)
    int tt = t;
    asm volatile("" : "+v"(tt));  // per-pivot compares stay local (no 64 hoisted masks)
    bsync<1>();
    const f4v r0 = S.bc[k & 1][lane & 15];
    const float v = K.k[k];
    const float p = __builtin_bit_cast(
        float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
    const float pinv = __builtin_amdgcn_rcpf(p);
    const float ng = -((tt == k) ? (1.0f - pinv) : v * pinv);
    if constexpr (k + 1 < KP) {  // unconditional past the last pivot (harmless): no branch to join
      const float la = fmaf(dpp_col<k + 1>(r0), ng, K.k[k + 1]);
      const float p1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, la), k + 1));
      reinterpret_cast<float *>(&S.bc[(k + 1) & 1][0])[tt] = (tt == k + 1) ? p1 + 1.0f : ((tt < k + 1) ? -la : la);
    }
    if constexpr (C60) {
      QL_DPP_GJ60(K.k, 0, r0, ng);
    } else {
      QL_DPP_GJ64(K.k, 0, r0, ng);
    }
    if (p > kGjExactPivot) K.k[k] = (tt == k) ? pinv : ng;  // column k exactly
  });
  bsync<1>();
}


// K0 / K2 table over (row step, column step); column NM is the zero row
// of padding lanes (cst = NM)
template <int W, int NM>
__device__ __forceinline__ void fill_k0k2(SrbdLds<W, NM> &S, int N, float Nf, int t) {
  for (int idx = t; idx < N * (NM + 1); idx += 64 * W) {
    const int sr = idx / (NM + 1), sc = idx - (NM + 1) * sr;
    float K0 = 0.0f, K2 = 0.0f;
    if (sc < N) k0k2((float)sr, (float)sc, Nf, K0, K2);
    S.k0k2[idx] = (f2v){K0, K2};
  }
}


// Two-wave form: the same transposed write, one pivot half per wave (the
// pivot column register is static inside each half), one s_barrier per
// pivot, the pivot value through LDS.
template <int H, int C2, int NM>
__device__ __forceinline__ void invert_w2_half(SrbdLds<2, NM> &S, int t, int nw, Row<2> &K) {
  int nc = __builtin_amdgcn_readfirstlane(nw);
#pragma unroll
  for (int kk = 0; kk < (H == 1 ? 4 * C2 : 64); ++kk) {
    asm volatile("" : "+s"(nc));
    if (kk >= nc) continue;  // block-uniform
    const int k = 64 * H + kk;
    const int buf = kk & 1;
    float *bcf = reinterpret_cast<float *>(&S.bc[buf][0]);
    int tt = t;
    asm volatile("" : "+v"(tt));
    const float v = K.k[k];
    bcf[tt] = (tt == k) ? v + 1.0f : ((tt < k) ? -v : v);
    S.colv[buf][tt] = v;  // the pivot A_kk for the other wave (no divergent store)
    __syncthreads();
    const float p = S.colv[buf][k];
    // chunk index from the per-pivot opaque copy: its LDS offset is not
    // hoisted to kernel entry (it was reloaded from scratch every pivot)
    const f4v r0 = S.bc[buf][tt & 15], r1 = S.bc[buf][16 + (tt & 15)];
    const float pinv = __builtin_amdgcn_rcpf(p);
    const float ng = -((tt == k) ? (1.0f - pinv) : v * pinv);
    QL_DPP_GJ64(K.k, 0, r0, ng);
    QL_HALF2(C2, QL_DPP_GJ12, QL_DPP_GJ24, QL_DPP_GJ36, QL_DPP_GJ60, QL_DPP_GJ64, K.k, 64, r1, ng);
    if (p > kGjExactPivot) K.k[k] = (tt == k) ? pinv : ng;  // column k exactly (invert_w1)
  }
}

template <int C2, int NM>
__device__ __forceinline__ void invert_w2(SrbdLds<2, NM> &S, int t, const int (&ncol)[2], Row<2> &K) {
  invert_w2_half<0, C2>(S, t, ncol[0], K);
  // the buffer parity restarts with the second half (its first pivot may
  // reuse the buffer of the first half's last one): all reads of that
  // buffer must be done before it is rewritten
  __syncthreads();
  invert_w2_half<1, C2>(S, t, ncol[1], K);
  __syncthreads();
}


// Occupancy (waves per SIMD, amdgpu_waves_per_eu) of each instantiation,
// every choice a same-call A/B:
//  * one-wave kernel, N <= kShortN: per-step LDS tables sized for N <= 10
//    (9 KB) and four waves per SIMD (128 VGPRs) -- all 4096 headline
//    instances resident from the first cycle (profiles/r3_occ_ab.txt);
//  * one-wave kernel, longer horizons: three waves (168 VGPRs, small spills
//    in the setup / refactor paths) above kSmallBatch instances, two waves
//    (186 VGPRs, spill-free) at or below it -- with few waves per SIMD the
//    tail of long instances dominates (profiles/r2ab_*, r2v_*);
//  * two-wave buckets C2 = 3 / 6 / 9 / 15: three waves; the C2 = 3 / 6
//    buckets at four waves for N <= 10 were 1.5 % faster but spilled inside
//    the ADMM loop (1.36 / 1.31 GB of scratch writes per mixed launch,
//    profiles/r3wt_*), so they are not instantiated;
//  * warm-started two-wave instances: one C2 = 15 instantiation at two waves.
constexpr int kShortN = 10;
constexpr int kShortWpe = 4;
constexpr int kW1Wpe = 3, kW1SmallWpe = 2;
constexpr int64_t kSmallBatch = 6144;
constexpr int kW2Wpe = 3, kW2WarmWpe = 2;

// WS: a warm-start mode (1 or 2) may be set.  The cold-start instantiation
// (the headline path) carries none of the warm / persistent-record code.
template <int W, bool WS, int NM, int C2 = 16>
__device__ __forceinline__ void srbd_solve_one(const SrbdArgs &a, SrbdLds<W, NM> &S, const int64_t b) {
  constexpr int NC = 64 * W, NQ = 16 * W;
  constexpr int NK = W == 1 ? (kW1Legs <= 20 ? 60 : 64) : 64 + 4 * C2;  // register columns of K in use
  const int t = threadIdx.x;
  const int wave = t >> 6, lane = t & 63;
  const int N = a.N;
  const float Nf = (float)N;
  const float dt = a.dt;
  const float dtm = dt / a.mass, dt2m = dt * dt / a.mass;

  // ---------------- 1. inputs -> LDS (one instance per block)
  if (t < 13) S.x0[t] = a.x0[b * 13 + t];
  if (t == 0) {  // static indices: kernel-argument arrays never indexed per lane
#pragma unroll
    for (int k = 0; k < 13; ++k) S.q2[k] = a.q2[k];
#pragma unroll
    for (int k = 0; k < 12; ++k) S.r2[k] = a.r2[k];
  }
  {
    const int nct = a.contacts_per_step ? 4 * N : 4;
    for (int k = t; k < 4 * N; k += NC)
      S.ct[k] = a.contacts[b * nct + (a.contacts_per_step ? k : (k & 3))] ? 1 : 0;
  }
  bsync<W>();

  // ---------------- 2. variable enumeration (integer, bit-exact): the stance
  // (step, leg) pairs, or every pair for the literal full QP
  if (wave == 0) {
    const bool s0 = (lane < 4 * N) && (a.literal || S.ct[lane]);
    const bool s1 = (64 + lane < 4 * N) && (a.literal || S.ct[64 + lane]);
    const uint64_t m0 = __ballot(s0), m1 = __ballot(s1);
    const uint64_t below = (1ull << lane) - 1ull;
    const int c0 = __popcll(m0);
    if (s0) S.legtab[__popcll(m0 & below)] = lane;
    if (s1) S.legtab[c0 + __popcll(m1 & below)] = 64 + lane;
    if (lane == 0) S.nlegs = c0 + __popcll(m1);
    if (lane <= N) {
      const int q = 4 * lane;
      const uint64_t l0 = q >= 64 ? ~0ull : ((1ull << q) - 1ull);
      const int q1 = q - 64;
      const uint64_t l1 = q1 <= 0 ? 0ull : ((1ull << q1) - 1ull);
      S.stepstart[lane] = __popcll(m0 & l0) + __popcll(m1 & l1);
    }
  }
  bsync<W>();
  const int nlegs = uni(S.nlegs);
  const int n = 3 * nlegs;
  if (nlegs < a.leg_lo || nlegs > a.leg_hi) return;  // the other launch's instance
  if (nlegs > (W == 1 ? kW1Legs : w2_bucket_legs(C2))) {  // uniform: the caller's max_stance_legs was too small
    if (t < 12) a.u0[b * 12 + t] = NAN;
    if (a.u)
      for (int k = t; k < 12 * N; k += NC) a.u[b * 12 * N + k] = NAN;
    if (t == 0) {
      if (a.status) a.status[b] = QLOCO_BAD_SIZE;
      if (a.iters) a.iters[b] = 0;
      if (a.rho_updates) a.rho_updates[b] = 0;
      if (a.obj) a.obj[b] = NAN;
    }
    return;
  }
  // persistent solver (warm_start == 2, A1RobotControl.cpp:556-578): the
  // record of this instance's last call (layout: QLOCO_SRBD_PERSIST_LEN)
  const int NP = 100 * N;
  float *prec = (WS && a.warm_start == 2) ? a.warm + b * (int64_t)(NP + 4) : nullptr;
  bool p_init = false, p_same = false;
  if (prec) {
    p_init = prec[NP + 1] > 0.5f;
    // literal full QP: the problem structure never changes (the reference's
    // Hessian pattern is contact-independent, ConvexMpc.cpp:211-215), so
    // every call after the first takes the update path; the stance-only
    // reduction re-initialises when its variable set changes
    int mism = 0;
    if (!a.literal)
      for (int k = t; k < 4 * N; k += 64 * W) mism |= (prec[96 * N + k] != 0.0f) != (S.ct[k] != 0);
    p_same = p_init && !__syncthreads_or(mism);
  }
  // valid columns per wave, from the stance-leg count (re-read from LDS at
  // each factorisation rather than kept live across the ADMM loop)
  auto col_counts = [&](int nl, int (&ncol)[W]) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      int lw = nl - kLegsPerWave * w;
      lw = lw < 0 ? 0 : (lw > kLegsPerWave ? kLegsPerWave : lw);
      ncol[w] = 3 * lw;
    }
  };
  // every valid column below 60: the 60-column DPP forms (uniform)
  const bool c60 = W == 1 && (kW1Legs <= 20 || 3 * nlegs <= 60);
  const int lslot = lane / 3;
  const int comp = lane - 3 * lslot;
  const bool valid = (lane < 63) && (kLegsPerWave * wave + lslot < nlegs);
  int step, leg;
  {
    const int pair = valid ? S.legtab[kLegsPerWave * wave + lslot] : 0;
    step = pair >> 2;
    leg = pair & 3;
  }
  S.cst[t] = valid ? step : NM;
  fill_k0k2<W>(S, N, Nf, t);

  // ---------------- 3. SRBD model terms (ConvexMpc.cpp:111-160, compute_grf :502-549)
  const float yaw = S.x0[2];
  const float cy = cosf(yaw), sy = sinf(yaw);
  // R = [[c,s,0],[-s,c,0],[0,0,1]] (A1RobotControl.cpp:506-508)
  const float R00 = cy, R01 = sy, R10 = -sy, R11 = cy;
  f4v lo, hi;
  {
    float Ii[3][3];
    const float *I = a.inertia;
    const float Rm[3][3] = {{R00, R01, 0.f}, {R10, R11, 0.f}, {0.f, 0.f, 1.f}};
    float RI[3][3], Iw[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        RI[r][c] = Rm[r][0] * I[c * 3 + 0] + Rm[r][1] * I[c * 3 + 1] + Rm[r][2] * I[c * 3 + 2];
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
    // this lane's B_d column (rows 6..8) and E = dt A_c B_d column (rows 0..2)
    const float *rf = a.feet + b * (a.feet_per_step ? 12 * N : 12) +
                      (a.feet_per_step ? 12 * step : 0) + 3 * leg;
    const float rx = rf[0], ry = rf[1], rz = rf[2];
    const float tv0 = comp == 0 ? 0.f : (comp == 1 ? -rz : ry);  // skew(r) e_comp (Utils.cpp:35-41)
    const float tv1 = comp == 0 ? rz : (comp == 1 ? 0.f : -rx);
    const float tv2 = comp == 0 ? -ry : (comp == 1 ? rx : 0.f);
    float ba[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) ba[r] = dt * (Ii[r][0] * tv0 + Ii[r][1] * tv1 + Ii[r][2] * tv2);
    lo = (f4v){ba[0], ba[1], ba[2], dt * (R00 * ba[0] + R01 * ba[1])};
    hi = (f4v){dt * (R10 * ba[0] + R11 * ba[1]), dt * ba[2], (float)step, (float)comp};
    if (!valid) {
      lo = (f4v)(0.0f);
      hi = (f4v){0.0f, 0.0f, 0.0f, -1.0f};
    }
    S.bv[t][0] = lo;
    S.bv[t][1] = hi;
  }
  const float r2v = valid ? S.r2[3 * leg + comp] : 0.0f;

  // ---------------- 4. gradient g = Bqp' Q (Aqp x0 - x_ref) (ConvexMpc.cpp:219-221)
  //     free response A_d^{i+1} x0 in closed form (A_c nilpotent)
  for (int idx = t; idx < 12 * N; idx += NC) {
    const int i = idx / 12, s = idx - 12 * i;
    const float k = (float)(i + 1);
    const float *x0 = S.x0;
    float xf;
    if (s < 3) {
      const float rw = s == 0 ? (R00 * x0[6] + R01 * x0[7]) : (s == 1 ? (R10 * x0[6] + R11 * x0[7]) : x0[8]);
      xf = x0[s] + k * dt * rw;
    } else if (s < 6) {
      xf = x0[s] + k * dt * x0[s + 6];
      if (s == 5) xf += 0.5f * k * (k - 1.0f) * dt * dt * x0[12];
    } else if (s < 9) {
      xf = x0[s];
    } else {
      xf = x0[s] + (s == 11 ? k * dt * x0[12] : 0.0f);
    }
    S.err[idx] = S.q2[s] * (xf - a.xref[b * 13 * N + 13 * i + s]);
  }
  // rows past the horizon stay zero for good (horizon_rows reads them)
  for (int idx = 12 * N + t; idx < 12 * NM; idx += NC) S.err[idx] = 0.0f;
  bsync<W>();
  row_scans<W>(S, N, false);
  bsync<W>();
  float qv = valid ? bqp_t<W>(S, step, comp, lo, hi, dtm, dt2m) : 0.0f;
  const float q_raw = qv;  // unscaled gradient entry (persistent record)
  // OSQP's update path runs scale_data on the new P with the PREVIOUS q in
  // place (osqp_update_P precedes osqp_update_lin_cost): the cost scale's
  // ||q|| comes from the previous call's gradient, scaled alongside
  float qsv = qv;
  if (p_same) qsv = valid ? prec[84 * N + 12 * step + 3 * leg + comp] : 0.0f;

  // ---------------- 5. constraint rows owned by this lane (ConvexMpc.cpp:47-59, :227-249)
  //  x lane: rows 0 [1,0, mu] in [0,inf), 1 [1,0,-mu] in (-inf,0]
  //  y lane: rows 2 [0,1, mu] in [0,inf), 3 [0,1,-mu] in (-inf,0]
  //  z lane: row 4 [0,0,1] in [fz_min, fz_max]; its slot 1 is an inert
  //  zero row with bounds [0,0] (stays z = y = 0), as are padding lanes.
  const bool xy = comp < 2;
  // A entries (ra0, ra1, rz0, rz1) of the two slots: LDS-resident from here on
  // (Ruiz scales them in place; registers would carry them across the setup)
  S.arz[t] = (f4v){valid ? 1.0f : 0.0f, (valid && xy) ? 1.0f : 0.0f, (valid && xy) ? a.mu : 0.0f,
                   (valid && xy) ? -a.mu : 0.0f};
  float rE0 = 1.0f, rE1 = 1.0f, Dr = 1.0f, cs = 1.0f;
  S.aux[0][t] = r2v;
  S.pair[t] = 4 * step + leg;

  Row<W> K;
  float cinv = 1.0f, rho = fminf(fmaxf(p_same ? prec[NP] : a.rho, 1e-6f), 1e6f), rvi = 1.0f / rho;
  bool eq0 = false;
#define RV0 (eq0 ? 1e3f * rho : rho)
#define RVI0 (eq0 ? 1e-3f * rvi : rvi)
  // leg block sigma I + A' diag(rho) A (3x3, leg-local); scaled A entries from LDS
  auto leg_block = [&](float &add0, float &add1, float &add2) {
    const f4v arz = S.arz[t];
    const f2v ra = {arz.x, arz.y}, rz = {arz.z, arz.w};
    const float rv0 = RV0, rv1 = rho;
    const float d_own = rv0 * ra.x * ra.x + rv1 * ra.y * ra.y;
    const float d_oz = rv0 * ra.x * rz.x + rv1 * ra.y * rz.y;
    const float d_zz = rv0 * rz.x * rz.x + rv1 * rz.y * rz.y;
    const float oz1 = lane_prev(d_oz), oz2 = lane_prev(oz1);
    const float zz1 = lane_prev(d_zz), zz2 = lane_prev(zz1);
    if (comp == 0) {
      add0 = d_own + a.sigma; add1 = 0.0f; add2 = d_oz;
    } else if (comp == 1) {
      add0 = 0.0f; add1 = d_own + a.sigma; add2 = d_oz;
    } else {
      add0 = oz2; add1 = oz1; add2 = d_own + zz1 + zz2 + a.sigma;
    }
    if (!valid) add0 = add1 = add2 = 0.0f;
  };

  // ---------------- 9. ADMM (OSQP osqp_solve) with its (re)factorisations
  float x = 0.0f;
  f2v z = (f2v)(0.0f), y = (f2v)(0.0f);
  const float alpha = a.alpha, oma = 1.0f - a.alpha, sigma = a.sigma;
  const int ctm = a.check_termination;
  const int interval = (a.adaptive_rho && a.rho_interval == 0)
                           ? (ctm ? 4 * ctm : 100)
                           : (a.adaptive_rho ? a.rho_interval : 0);
  int status = QLOCO_MAX_ITER, iter = 0;
  float px = 0.0f;  // scaled (P x)_v of the last residual evaluation
  bool first = true;
  int rho_updates = 0;

  // residual norms (OSQP update_info), all lanes participate.
  //  o[0] ||E^-1(Ax-z)||  o[1] ||E^-1 z||  o[2] ||E^-1 A x||  o[3] ||D^-1 rd||
  //  o[4] ||D^-1 A'y||    o[5] ||D^-1 P x||
  //  r[0..5] the scaled ||Ax-z||, ||z||, ||Ax||, ||rd||, ||A'y||, ||Px|| (rho estimate)
  auto residuals = [&](float (&o)[6], float (&r)[6], bool want_r) {
    const float Drl = S.Dc[t];
    S.xs[t] = valid ? x * Drl : 0.0f;
    bsync<W>();
    const f4v blo = S.bv[t][0], bhi = S.bv[t][1];
    const float pxo = p_times_x<W>(S, N, valid, (int)bhi.z, comp, blo, bhi, S.aux[0][t], x * Drl,
                                   dtm, dt2m);
    const float Dinv = __builtin_amdgcn_rcpf(Drl);
    const f2v Einv = {__builtin_amdgcn_rcpf(S.aux[1][t]), __builtin_amdgcn_rcpf(S.aux[2][t])};
    const f4v arz = S.arz[t];
    const f2v ra = {arz.x, arz.y}, rz = {arz.z, arz.w};
    const float qv = S.qs[t];
    px = cs * Drl * pxo;
    const float n1 = lane_next(x), n2 = lane_next(n1);
    const float xz = comp == 0 ? n2 : (comp == 1 ? n1 : x);
    const f2v ay = ra * y, az = rz * y;
    const float ay_z = az.x + az.y;
    const float p1 = lane_prev(ay_z), p2 = lane_prev(p1);
    const float aty = valid ? ((ay.x + ay.y) + (comp == 2 ? (p1 + p2) : 0.0f)) : 0.0f;
    const float rd = valid ? (qv + px + aty) : 0.0f;
    const f2v ax = ra * x + rz * xz;
    const f2v rp = ax - z;
    const f2v erp = Einv * rp, ez = Einv * z, eax = Einv * ax;
    o[0] = fmaxf(fabsf(erp.x), fabsf(erp.y));
    o[1] = fmaxf(fabsf(ez.x), fabsf(ez.y));
    o[2] = fmaxf(fabsf(eax.x), fabsf(eax.y));
    o[3] = fabsf(Dinv * rd);
    o[4] = fabsf(Dinv * aty);
    o[5] = fabsf(Dinv * px);
    bmax<W, 6>(o, S.red);
    if (want_r) {
      r[0] = fmaxf(fabsf(rp.x), fabsf(rp.y));
      r[1] = fmaxf(fabsf(z.x), fabsf(z.y));
      r[2] = fmaxf(fabsf(ax.x), fabsf(ax.y));
      r[3] = fabsf(rd);
      r[4] = fabsf(aty);
      r[5] = fabsf(px);
      bmax<W, 6>(r, S.red);
    }
  };

  // One code path for the first factorisation and every adaptive-rho
  // refactorisation: closed-form P row -> (first: Ruiz) -> K = cs D P D +
  // leg blocks -> K^-1 -> ADMM blocks.  Each piece is emitted once (the
  // kernel is instruction-cache bound: DESIGN.md §3d).
  for (;;) {
    {  // closed-form P row, regenerated for every factorisation
      const f4v blo = S.bv[t][0], bhi = S.bv[t][1];
      const PCoef pc = p_coef<W>(S, blo, bhi, comp, valid, dtm, dt2m);
      gen_p_row<W, C2>(S, pc, t, valid, (int)bhi.z, comp, S.aux[0][t], K);
    }
    if (first) {
      // ---------------- 7. modified Ruiz equilibration (OSQP scaling.c); K
      // keeps the unscaled P, row norms of the scaled P = cs D P D come from
      // the DPP-fanned D chunk
      float cnP = 0.0f;
#pragma unroll
      for (int c = 0; c < NK; ++c) cnP = fmaxf(cnP, fabsf(KE(K, c)));
      const int n_r = 3 * uni(S.nlegs);  // re-read: 1/n stays out of the loop-live set
      const float inv_n = 1.0f / (float)(n_r > 0 ? n_r : 1);
      for (int it = 0; it < a.scaling; ++it) {
        asm volatile("" ::: "memory");  // re-read the entries (not forwarded in registers)
        const f4v arz0 = S.arz[t];
        float ra0 = arz0.x, ra1 = arz0.y, rz0 = arz0.z, rz1 = arz0.w;
        float cnA = fmaxf(fabsf(ra0), fabsf(ra1));
        const float zmax = fmaxf(fabsf(rz0), fabsf(rz1));
        const float zm1 = lane_prev(zmax), zm2 = lane_prev(zm1);
        if (comp == 2) cnA = fmaxf(cnA, fmaxf(zm1, zm2));
        // v_rsq_f32 (1 ulp): the Ruiz factors are heuristics, not exact quantities
        const float Dt = valid ? __builtin_amdgcn_rsqf(limit_scaling(fmaxf(cnP, cnA))) : 1.0f;
        const float Et0 = valid ? __builtin_amdgcn_rsqf(limit_scaling(fmaxf(fabsf(ra0), fabsf(rz0)))) : 1.0f;
        const float Et1 = (valid && xy) ? __builtin_amdgcn_rsqf(limit_scaling(fmaxf(fabsf(ra1), fabsf(rz1)))) : 1.0f;
        // z lane's D for the mu entries of the x/y lanes' rows
        const float Dn1 = lane_next(Dt), Dn2 = lane_next(Dn1);
        const float Dz = comp == 0 ? Dn2 : (comp == 1 ? Dn1 : Dt);
        ra0 *= Et0 * Dt;
        ra1 *= Et1 * Dt;
        rz0 *= Et0 * Dz;
        rz1 *= Et1 * Dz;
        S.arz[t] = (f4v){ra0, ra1, rz0, rz1};
        rE0 *= Et0;
        rE1 *= Et1;
        qv *= Dt;
        qsv *= Dt;
        Dr *= Dt;
        const int buf = it & 1;
        reinterpret_cast<float *>(&S.bc[buf][0])[t] = Dr;
        bsync<W>();
        float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f, t0, t1, t2, t3;
        {
          const f4v d0 = S.bc[buf][lane & 15];
          if (W == 1 && c60) {  // padding columns: K_rc = 0 on valid rows
            QL_DPP_ABSMAX60(m0, m1, m2, m3, t0, t1, t2, t3, d0, K.k, 0);
          } else {
            QL_DPP_ABSMAX64(m0, m1, m2, m3, t0, t1, t2, t3, d0, K.k, 0);
          }
          if constexpr (W == 2) {
            const f4v d1 = S.bc[buf][16 + (lane & 15)];
            QL_HALF2(C2, QL_DPP_ABSMAX12, QL_DPP_ABSMAX24, QL_DPP_ABSMAX36, QL_DPP_ABSMAX60, QL_DPP_ABSMAX64, m0, m1,
                     m2, m3, t0, t1, t2, t3, d1, K.k, 64);
          }
        }
        // row norm of D P D after this pass (without the running cost scale)
        const float cn2 = Dr * fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
        // cost scaling: mean column norm of P (= row norm, P symmetric) vs ||q||_inf
        const float sumP = bsum<W>(valid ? cn2 : 0.0f, S.red);
        float qm[1] = {valid ? fabsf(qsv) : 0.0f};
        bmax<W, 1>(qm, S.red);
        const float meanP = cs * sumP * inv_n;
        // v_rcp_f32 (1 ulp), like the rsq above: a heuristic factor
        const float ctc = __builtin_amdgcn_rcpf(limit_scaling(fmaxf(meanP, limit_scaling(qm[0]))));
        qv *= ctc;
        qsv *= ctc;
        cs *= ctc;
        cnP = cn2 * cs;
      }
      cinv = 1.0f / cs;
      // fz in [fz_min * c, fz_max * c] (ConvexMpc.cpp:237, :242): c = 1 on every
      // stance pair, 0 on the swing pairs the literal full QP keeps (computed
      // here, not at entry: kept live across the setup they spilled)
      const float cflag = valid ? (float)S.ct[S.pair[opaque_tid()]] : 0.0f;
      const float rl0 = !valid ? 0.0f : (xy ? 0.0f : a.fz_min * cflag);
      const float ru0 = !valid ? 0.0f : (xy ? INFINITY : a.fz_max * cflag);
      const float lh0 = rl0 * rE0, uh0 = ru0 * rE0;
      // slot 1: (-inf, 0] on x/y lanes (E scaling keeps 0 and inf), inert [0, 0] elsewhere
      const float lh1 = (valid && xy) ? -INFINITY : 0.0f, uh1 = 0.0f;
      // OSQP set_rho_vec: every SRBD row is a two-sided or one-sided inequality
      // (rho) except a z row with fz_max - fz_min < RHO_TOL (equality, 1e3 rho);
      // no row is loose.  The inert slot-1 rows have a zero A row, so their rho
      // never matters -- rho vector = (eq0 ? 1e3 rho : rho, rho).
      eq0 = valid && !xy && (uh0 - lh0 < 1e-4f);
      S.Dc[t] = valid ? Dr : 1.0f;
      S.aux[1][t] = rE0;
      S.aux[2][t] = rE1;
      S.zb[t] = (f4v){lh0, uh0, lh1, uh1};
      // ||D^-1 q||_inf and ||q||_inf (scaled) are constant over the iterations
      float qn[2] = {fabsf(qv / Dr), fabsf(qv)};
      bmax<W, 2>(qn, S.red);
      if (t == 0) {
        S.qn[0] = qn[0];
        S.qn[1] = qn[1];
      }
      S.qs[t] = qv;
      bsync<W>();
    }
    // ---------------- 8. K = cs D P D + sigma I + A' rho A, inverse in registers
    {
      float add0, add1, add2;
      leg_block(add0, add1, add2);
      const float dg = finalize_row<W, C2>(S, t, t - comp, cs * S.Dc[t], add0, add1, add2, c60, K);
      int ncol[W];
      col_counts(uni(S.nlegs), ncol);
      if constexpr (W == 1) {
        (void)dg;
        if (c60) {
          invert_w1<true>(S, t, ncol[0], K);
        } else {
          invert_w1<false>(S, t, ncol[0], K);
        }
      } else {
        (void)dg;
        invert_w2<C2>(S, t, ncol, K);
      }
    }
    if (first) {
      first = false;
      // record offsets from an opaque thread copy: no per-lane record address
      // is kept live from the entry's reads of the record
      const int tf = opaque_tid(), pf = S.pair[tf], lf = tf & 63, cf = lf - 3 * (lf / 3);
      const int vidx = 12 * (pf >> 2) + 3 * (pf & 3) + cf, rbase = 20 * (pf >> 2) + 5 * (pf & 3) + 2 * cf;
      if (p_same) {
        // live workspace (osqp_solve without cold start): the scaled
        // iterates of the last call as they are
        x = valid ? prec[vidx] : 0.0f;
        z.x = valid ? prec[12 * N + rbase] : 0.0f;
        z.y = (valid && xy) ? prec[12 * N + rbase + 1] : 0.0f;
        y.x = valid ? prec[32 * N + rbase] : 0.0f;
        y.y = (valid && xy) ? prec[32 * N + rbase + 1] : 0.0f;
      } else if (WS && (a.warm_start == 1 || p_init)) {
        // osqp_warm_start from the unscaled x | y: the caller's buffer
        // (warm_start 1) or, for a persistent solver whose stance set
        // changed, the record's last solution (OsqpEigen re-initialisation
        // + setPrimal/DualVariable)
        const float *wx = a.warm_start == 1 ? a.warm + b * (32 * N) : prec + 52 * N;
        const float *wy = wx + 12 * N;
        x = valid ? wx[vidx] / Dr : 0.0f;
        y.x = valid ? wy[rbase] / rE0 * cs : 0.0f;
        y.y = (valid && xy) ? wy[rbase + 1] / rE1 * cs : 0.0f;
        const float n1 = lane_next(x), n2 = lane_next(n1);
        const float xz = comp == 0 ? n2 : (comp == 1 ? n1 : x);
        const f4v arz = S.arz[t];
        z = (f2v){arz.x, arz.y} * x + (f2v){arz.z, arz.w} * xz;
      }
    }
    bool refactor = false;

    // Iterations run in event-free blocks up to the next termination check,
    // adaptive-rho point or max_iter, so the hot loop carries no modulo tests;
    // the residual evaluation after a block is the only one in the kernel
    // (checks, rho estimates and the final max_iter status share it).
    for (;;) {
      if (iter < a.max_iter) {
      int next = a.max_iter;
      if (ctm) next = min(next, (iter / ctm + 1) * ctm);
      if (interval) next = min(next, (iter / interval + 1) * interval);
      // block-local copies: dead again in the cold paths below
      const f4v arz = S.arz[t];
      const f2v ra = {arz.x, arz.y}, rz = {arz.z, arz.w};
      const float qv = S.qs[t];
      const f2v rv = {RV0, rho}, rvi2 = {RVI0, rvi};
      const float m2 = comp == 2 ? 1.0f : 0.0f;
      // C60: n <= 60, columns 60..63 are identity padding (K^-1 entries 0)
      // W = 2: CH = chunks of the second row half (9 / 15 / 16)
      auto run_block = [&](auto c60_tag, auto ch_tag) {
      constexpr bool C60 = decltype(c60_tag)::value;
      constexpr int CH = decltype(ch_tag)::value;
      for (; iter < next; ++iter) {
        // compiler-only barrier: LDS-resident tables (bv, Dc, zb, ...) are
        // re-read where used instead of being hoisted into loop-live registers
        asm volatile("" ::: "memory");
        const f4v bnd = S.zb[t];  // projection bounds: LDS, issued early, not loop-carried
        // rhs = sigma x_prev - q + A'(rho z_prev - y)   (compute_rhs); padding
        // lanes have zero A rows and q, so their rhs is 0 without a select
        const f2v w = __builtin_elementwise_fma(rv, z, -y);
        const f2v aw = ra * w, zw = rz * w;
        const float tz = zw.x + zw.y;
        float rhs = fmaf(sigma, x, (aw.x + aw.y) - qv);
        // z lane: += tz[l-1] + tz[l-2] (its leg's x and y lanes), as two
        // DPP-fused ops: u = tz[l-1] + tz[l], rhs += m2 * u[l-1]
        {
          float u;
          asm("s_nop 1\n\t"
              "v_add_f32_dpp %0, %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "s_nop 1\n\t"
              "v_fmac_f32_dpp %1, %0, %3 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
              : "=&v"(u), "+v"(rhs)
              : "v"(tz), "v"(m2));
        }
        // one wave's LDS operations complete in order: W = 1 needs no double buffer
        const int buf = W == 1 ? 0 : (iter & 1);
        reinterpret_cast<float *>(&S.bc[buf][0])[t] = rhs;
        bsync<W>();
        // x_tilde = K^-1 rhs: one 16-byte LDS chunk per lane, DPP row_newbcast
        // fans it out to the register-resident row (qloco_dpp.inc)
        float xt;
        {
          const f4v r0 = S.bc[buf][lane & 15];
          if constexpr (W == 1) {
            // two accumulator chains (four measured no faster)
            float acc0, acc1;
            if constexpr (C60) {
              QL_DPP_MATVEC60_2(acc0, acc1, r0, K.k, 0);
            } else {
              QL_DPP_MATVEC64_2(acc0, acc1, r0, K.k, 0);
            }
            xt = acc0 + acc1;
          } else {
            float acc0, acc1, acc2, acc3;
            QL_DPP_MATVEC64(acc0, acc1, acc2, acc3, r0, K.k, 0);
            if constexpr (W == 2) {
              const f4v r1 = S.bc[buf][16 + (lane & 15)];
              if constexpr (CH == 3) {
                QL_DPP_MATVEC12_ACC(acc0, acc1, acc2, acc3, r1, K.k, 64);
              } else if constexpr (CH == 6) {
                QL_DPP_MATVEC24_ACC(acc0, acc1, acc2, acc3, r1, K.k, 64);
              } else if constexpr (CH == 9) {
                QL_DPP_MATVEC36_ACC(acc0, acc1, acc2, acc3, r1, K.k, 64);
              } else if constexpr (CH == 15) {
                QL_DPP_MATVEC60_ACC(acc0, acc1, acc2, acc3, r1, K.k, 64);
              } else {
                QL_DPP_MATVEC64_ACC(acc0, acc1, acc2, acc3, r1, K.k, 64);
              }
            }
            xt = (acc0 + acc1) + (acc2 + acc3);
          }
        }
        // x / y lanes take their leg's z lane (2 / 1 lanes up); z lanes have
        // rz = 0, so their pick is irrelevant
        const float n1 = lane_next(xt), n2 = lane_next(n1);
        const float xtz = comp == 0 ? n2 : n1;
        // update_x / update_z / update_y (relaxation alpha, projection on [l, u])
        x = fmaf(alpha, xt, oma * x);
        const f2v zt = __builtin_elementwise_fma(rz, (f2v)(xtz), ra * xt);
        const f2v zr = __builtin_elementwise_fma((f2v)(alpha), zt, oma * z);
        const f2v v = __builtin_elementwise_fma(y, rvi2, zr);
        const f2v zn = {__builtin_amdgcn_fmed3f(v.x, bnd.x, bnd.y),
                        __builtin_amdgcn_fmed3f(v.y, bnd.z, bnd.w)};
        y = __builtin_elementwise_fma(rv, zr - zn, y);
        z = zn;
      }
      };
      if constexpr (W == 1) {
        if (c60) {
          run_block(std::true_type{}, std::integral_constant<int, 16>{});
        } else {
          run_block(std::false_type{}, std::integral_constant<int, 16>{});
        }
      } else {
        run_block(std::false_type{}, std::integral_constant<int, C2>{});
      }
      }
      // OSQP: termination check every check_termination iterations, rho
      // adaptation every interval; past max_iter the status is "solved
      // inaccurate" or "max_iter reached" from the same residuals (an
      // adaptation at the last iteration keeps its rho for the record, its
      // refactorisation would be dead work and is skipped)
      const bool fin = iter >= a.max_iter;
      const bool can_check = ctm && iter > 0 && (iter % ctm == 0);
      const bool do_rho = interval && iter > 0 && (iter % interval == 0);
      if (!(can_check || do_rho || fin)) continue;
      float o[6], r[6];
      residuals(o, r, do_rho);
      const float pri_res = o[0], dua_res = cinv * o[3];
      const float qn0 = S.qn[0], qn1 = S.qn[1];  // set at the first factorisation, behind its barrier
      if (can_check) {
        const float eps_p = a.eps_abs + a.eps_rel * fmaxf(o[1], o[2]);
        const float eps_d = a.eps_abs + a.eps_rel * cinv * fmaxf(fmaxf(qn0, o[4]), o[5]);
        if (pri_res < eps_p && dua_res < eps_d) {
          status = QLOCO_OK;
          break;
        }
      }
      if (do_rho) {  // compute_rho_estimate + adapt_rho
        const float pn = r[0] / (fmaxf(r[1], r[2]) + 1e-30f);
        const float dn = r[3] / (fmaxf(fmaxf(qn1, r[4]), r[5]) + 1e-30f);
        float rho_new = rho * sqrtf(pn / (dn + 1e-30f));
        rho_new = fminf(fmaxf(rho_new, 1e-6f), 1e6f);
        if (rho_new > rho * a.rho_tol || rho_new < rho / a.rho_tol) {
          rho = rho_new;
          rvi = 1.0f / rho;
          rho_updates++;
          if (!fin) {
            refactor = true;
            break;
          }
        }
      }
      if (fin) {  // max_iter reached (OSQP: solved inaccurate or max_iter)
        // laundered: 10 eps is otherwise hoisted into two loop-live VGPRs
        float e_abs = a.eps_abs, e_rel = a.eps_rel;
        asm volatile("" : "+v"(e_abs), "+v"(e_rel));
        const float ep = 10.f * e_abs + 10.f * e_rel * fmaxf(o[1], o[2]);
        const float ed = 10.f * e_abs + 10.f * e_rel * cinv * fmaxf(fmaxf(qn0, o[4]), o[5]);
        // block-uniform: an SGPR, not a VGPR kept live to the outputs
        status = __builtin_amdgcn_readfirstlane((pri_res < ep && dua_res < ed) ? QLOCO_SOLVED_INACCURATE
                                                                                 : QLOCO_MAX_ITER);
        break;
      }
    }
    if (!refactor) break;
  }

  // ---------------- 10. outputs: unscale, objective, scatter to leg slots
  const int to = opaque_tid();  // the thread index (and its byte offsets) re-derived here
  const float Dr_o = S.Dc[to];
  const int pr_o = S.pair[to];
  const int step_o = pr_o >> 2, leg_o = pr_o & 3;
  const float xu = valid ? x * Dr_o : 0.0f;
  const float objp = bsum<W>(valid ? cinv * (0.5f * x * px + S.qs[to] * x) : 0.0f, S.red);
  const bool bad = !isfinite(objp);
  if (bad) status = QLOCO_NAN;
  if (a.u) {  // full solution (world frame), swing forces exactly 0
    float *uo = a.u + b * 12 * N;
    for (int k = to; k < 12 * N; k += NC) uo[k] = 0.0f;
    __syncthreads();
    if (valid) uo[12 * step_o + 3 * leg_o + comp] = bad ? NAN : xu;
  }
  // u0: step-0 forces; optional body frame R' u (A1RobotControl.cpp:596-599)
  S.xs[to] = xu;
  bsync<W>();
  if (to < 12) {
    const int lg = to / 3, cp = to - 3 * lg;
    float f0 = 0.f, f1 = 0.f, f2 = 0.f;
    for (int p = 0; p < S.stepstart[1]; ++p) {
      if ((S.legtab[p] & 3) == lg) {
        const int vb = 64 * (p / kLegsPerWave) + 3 * (p % kLegsPerWave);
        f0 = S.xs[vb];
        f1 = S.xs[vb + 1];
        f2 = S.xs[vb + 2];
      }
    }
    float o = cp == 0 ? f0 : (cp == 1 ? f1 : f2);
    if (a.output_frame == 1) {  // R^T f with R = [[c,s,0],[-s,c,0],[0,0,1]]
      // the rotation re-derived from the yaw in LDS (not kept live since section 3)
      const float oy = S.x0[2], oc = cosf(oy), os = sinf(oy);
      o = cp == 0 ? (oc * f0 - os * f1) : (cp == 1 ? (os * f0 + oc * f1) : f2);
    }
    a.u0[b * 12 + to] = bad ? NAN : o;
  }
  if (prec) {  // the persistent record for the next call
    for (int k = to; k < NP + 4; k += NC) prec[k] = 0.0f;
    __syncthreads();
    if (valid) {
      const int vidx = 12 * step_o + 3 * leg_o + comp, rbase = 20 * step_o + 5 * leg_o + 2 * comp;
      prec[vidx] = x;
      prec[52 * N + vidx] = xu;
      prec[84 * N + vidx] = q_raw;
      prec[12 * N + rbase] = z.x;
      prec[32 * N + rbase] = y.x;
      prec[64 * N + rbase] = cinv * S.aux[1][to] * y.x;
      if (xy) {
        prec[12 * N + rbase + 1] = z.y;
        prec[32 * N + rbase + 1] = y.y;
        prec[64 * N + rbase + 1] = cinv * S.aux[2][to] * y.y;
      }
    }
    for (int k = to; k < 4 * N; k += NC) prec[96 * N + k] = S.ct[k] ? 1.0f : 0.0f;
    if (to == 0) {
      prec[NP] = rho;
      prec[NP + 1] = 1.0f;
    }
  }
  if (WS && a.warm_start == 1) {
    const int nu = 12 * N, ncn = 20 * N;
    float *wx = a.warm + b * (nu + ncn);
    float *wy = wx + nu;
    for (int k = to; k < nu + ncn; k += NC) wx[k] = 0.0f;
    __syncthreads();
    if (valid) {
      wx[12 * step_o + 3 * leg_o + comp] = xu;
      const int rbase = 20 * step_o + 5 * leg_o + 2 * comp;
      wy[rbase] = cinv * S.aux[1][to] * y.x;
      if (xy) wy[rbase + 1] = cinv * S.aux[2][to] * y.y;
    }
  }
  if (to == 0) {
    if (a.status) a.status[b] = status;
    if (a.iters) a.iters[b] = iter;
    if (a.rho_updates) a.rho_updates[b] = rho_updates;
    if (a.obj) a.obj[b] = objp;
  }
}

// One instance per workgroup: instance list[blockIdx] (or blockIdx) for
// list positions below the device-side count (or the batch).
template <int W, int WPE, bool WS, int NM = kMaxN, int C2 = 16>
__global__ __launch_bounds__(64 * W)
__attribute__((amdgpu_waves_per_eu(WPE)))
void srbd_admm_kernel(const SrbdArgs a) {
  __shared__ __attribute__((aligned(16))) SrbdLds<W, NM> S;
  const int64_t i = blockIdx.x;
  if (i >= (a.count ? (int64_t)*a.count : a.batch)) return;
  srbd_solve_one<W, WS, NM, C2>(a, S, a.list ? (int64_t)a.list[i] : i);
}

// Kernel classes by stance-leg count: 0 one wave (<= kW1Legs), 1..4 two
// waves in the column buckets C2 = 3 / 6 / 9 / 15 (<= 25 / 29 / 33 / 41
// legs), 5..7 the wide kernel at half widths 96 / 112 / 120 (<= 64 / 74 /
// 80 legs; qloco_srbd_big.inc).  Warm-started launches use the widest
// bucket of each family (one warm instantiation per family).
constexpr int kSrbdClasses = 8;
constexpr int kBigLegs64 = 64, kBigLegs74 = 74;  // = big_bucket_legs(96 / 112)
__host__ __device__ constexpr int srbd_class_of(int legs, bool ws) {
  return legs <= kW1Legs ? 0
         : legs <= w2_bucket_legs(15)
             ? (ws ? 4
                   : (legs <= w2_bucket_legs(3) ? 1
                      : legs <= w2_bucket_legs(6) ? 2 : legs <= w2_bucket_legs(9) ? 3 : 4))
             : (ws ? 7 : (legs <= kBigLegs64 ? 5 : legs <= kBigLegs74 ? 6 : 7));
}

// Class of every instance (capped at the top class the launch admits),
// appended to that class's list: one ballot per class and wave, one atomic
// per wave and class (list order within a wave is instance order).
__global__ __launch_bounds__(256) void srbd_classify_kernel(const SrbdArgs a, int top, int *lists,
                                                            int64_t cap, int *counts) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int N = a.N;
  int cls = -1;
  if (b < a.batch) {
    int legs = 0;
    if (a.literal) {
      legs = 4 * N;
    } else if (a.contacts_per_step) {
      const uint8_t *c = a.contacts + b * 4 * N;
      for (int k = 0; k < 4 * N; ++k) legs += c[k] != 0;
    } else {
      for (int k = 0; k < 4; ++k) legs += a.contacts[b * 4 + k] != 0;
      legs *= N;
    }
    cls = srbd_class_of(legs, a.warm_start != 0);
    cls = cls > top ? top : cls;
  }
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int c = 0; c <= top; ++c) {
    const uint64_t m = __ballot(cls == c);
    if (!m) continue;
    int base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&counts[c], __popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (cls == c) lists[(int64_t)c * cap + base + __popcll(m & below)] = (int)b;
  }
}

}  // namespace qloco

#include "qloco_srbd_big.inc"

using namespace qloco;

extern "C" void qloco_srbd_spec_default(qloco_srbd_spec *s) {
  memset(s, 0, sizeof(*s));
  s->horizon = 10;
  s->feet_per_step = 0;
  s->contacts_per_step = 1;
  s->output_frame = 0;
  s->dt = 0.0025f;
  s->mass = 12.0f;  // gait::mass (robot_const_para_config.cpp:32)
  // Momentum_sum = 2 x Go1 trunk inertia (servo.cpp:375-377, go1.urdf:435)
  const float I[9] = {2 * 0.0168352186f, 2 * 0.0004636141f, 2 * 0.0002367952f,
                      2 * 0.0004636141f, 2 * 0.0656071082f, 2 * 3.6671e-05f,
                      2 * 0.0002367952f, 2 * 3.6671e-05f,   2 * 0.0742720659f};
  for (int k = 0; k < 9; ++k) s->inertia[k] = I[k];
  // gazebo_a1_mpc.yaml weights
  const float q[13] = {20, 10, 1, 0, 0, 420, 0.05f, 0.05f, 0.05f, 30, 30, 10, 0};
  for (int k = 0; k < 13; ++k) s->q_weights[k] = q[k];
  for (int k = 0; k < 12; ++k) s->r_weights[k] = 1e-7f;
  s->mu = 0.3f;
  s->fz_min = 0.0f;
  s->fz_max = 180.0f;
  // OSQP v0.6 defaults
  s->rho = 0.1f;
  s->sigma = 1e-6f;
  s->alpha = 1.6f;
  s->eps_abs = 1e-3f;
  s->eps_rel = 1e-3f;
  s->max_iter = 4000;
  s->check_termination = 25;
  s->scaling = 10;
  s->adaptive_rho = 1;
  s->adaptive_rho_interval = 0;
  s->adaptive_rho_tolerance = 5.0f;
  s->warm_start = 0;
  s->polish = 0;
}


// Scratch of the class dispatch: the per-class instance lists (`cap` entries
// each), their counters, three side streams and the fork / join events --
// one set per (device, caller stream), so calls on different streams or
// threads never share lists, counters or events (two calls on ONE stream
// are ordered by it), and a capture on one stream never pulls another
// caller's side streams into its graph.  The sets are bounded: at most
// kScratchSets live ones, the least recently used beyond that is released
// (its last class launch waited for by an event first), so callers that
// spin up short-lived streams do not leak streams, events or memory.  A set
// that ever served a stream capture is different: the graph baked its list
// and counter pointers in, so its memory is pinned for the life of the
// process (its streams and events are still released) -- as are the lists
// it outgrew.  Growing inside a stream capture is refused (QLOCO_ERR_ARG):
// run the largest batch once before capturing.  A captured
// graph shares its set with later eager calls on the capture stream: replay
// it ordered against them (graph capture).
struct SrbdScratch {
  int *lists = nullptr;
  int *counts = nullptr;
  int64_t cap = 0;
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  hipEvent_t fork = nullptr, join[3] = {nullptr, nullptr, nullptr};
  hipEvent_t done = nullptr;  // recorded on the caller's stream after the last eager use
  bool done_recorded = false;
  bool captured = false;  // served a stream capture: memory pinned
  uint64_t last_use = 0;
};
constexpr size_t kScratchSets = 8;
static std::mutex g_srbd_scratch_mu;
static std::map<std::pair<int, hipStream_t>, SrbdScratch> g_srbd_scratch;
static std::mutex g_srbd_pinned_mu;        // guards g_srbd_pinned (released sets push to it unlocked)
static std::vector<void *> g_srbd_pinned;  // memory a captured graph may still read
static uint64_t g_srbd_tick = 0;

// Releases a set that is no longer in g_srbd_scratch (the caller does not
// hold g_srbd_scratch_mu: the wait for the set's last launch blocks no other
// thread's class dispatch).  The calls run in this thread's relaxed capture
// mode, so a stream capture another thread runs in global mode
// (torch.cuda.graph's default) is not invalidated by them (INTEGRATION.md,
// graph capture).
static void srbd_release(SrbdScratch &s) {
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
  if (s.done_recorded) (void)hipEventSynchronize(s.done);
  for (int k = 0; k < 3; ++k) {
    if (s.side[k]) (void)hipStreamDestroy(s.side[k]);
    if (s.join[k]) (void)hipEventDestroy(s.join[k]);
  }
  if (s.fork) (void)hipEventDestroy(s.fork);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.captured) {
    std::lock_guard<std::mutex> lk(g_srbd_pinned_mu);
    g_srbd_pinned.push_back(s.lists);
    g_srbd_pinned.push_back(s.counts);
  } else {
    if (s.lists) (void)hipFree(s.lists);
    if (s.counts) (void)hipFree(s.counts);
  }
  if (swapped) (void)hipThreadExchangeStreamCaptureMode(&mode);
  s = SrbdScratch();
}

// Live scratch sets and pinned allocations (tests: the bound holds).
extern "C" int qloco_srbd_scratch_sets(int32_t *pinned) {
  std::lock_guard<std::mutex> lk(g_srbd_scratch_mu);
  if (pinned) {
    std::lock_guard<std::mutex> lp(g_srbd_pinned_mu);
    *pinned = (int32_t)g_srbd_pinned.size();
  }
  return (int)g_srbd_scratch.size();
}

// Caller holds g_srbd_scratch_mu for the whole enqueue sequence (counter
// reset, classification, class launches, the done event): two threads
// sharing one stream must not interleave their sequences on the shared
// counters.  A least-recently-used set evicted to make room is moved out of
// the map into *victim; the caller releases it after dropping the lock.
static int srbd_scratch(int64_t batch, hipStream_t st, bool capturing, SrbdScratch **out,
                        SrbdScratch *victim) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return QLOCO_ERR_DEVICE;
  const auto key = std::make_pair(dev, st);
  auto it = g_srbd_scratch.find(key);
  if (it == g_srbd_scratch.end()) {
    if (capturing) {
      set_last_error("qloco_srbd_solve_ex: class-dispatch scratch must be sized before stream "
                     "capture (run the largest batch once on this stream first)",
                     hipErrorStreamCaptureUnsupported);
      return QLOCO_ERR_ARG;
    }
    // a new set is built completely before it enters the map: a failure part
    // way leaves nothing half-initialised behind (the next call retries)
    SrbdScratch fresh;
    bool ok = hipMalloc(&fresh.counts, 8 * sizeof(int)) == hipSuccess;
    for (int k = 0; ok && k < 3; ++k) {
      ok = hipStreamCreateWithFlags(&fresh.side[k], hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&fresh.join[k], hipEventDisableTiming) == hipSuccess;
    }
    ok = ok && hipEventCreateWithFlags(&fresh.fork, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&fresh.done, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      srbd_release(fresh);
      return QLOCO_ERR_DEVICE;
    }
    // bound the live sets: the least recently used one leaves the map (the
    // caller releases it after unlocking)
    if (g_srbd_scratch.size() >= kScratchSets) {
      auto lru = g_srbd_scratch.begin();
      for (auto j = g_srbd_scratch.begin(); j != g_srbd_scratch.end(); ++j)
        if (j->second.last_use < lru->second.last_use) lru = j;
      *victim = lru->second;
      g_srbd_scratch.erase(lru);
    }
    it = g_srbd_scratch.emplace(key, fresh).first;
  }
  SrbdScratch &s = it->second;
  if (batch > s.cap) {
    if (capturing) {
      set_last_error("qloco_srbd_solve_ex: class-dispatch scratch must be sized before stream "
                     "capture (run the largest batch once on this stream first)",
                     hipErrorStreamCaptureUnsupported);
      return QLOCO_ERR_ARG;
    }
    const int64_t cap = batch < 4096 ? 4096 : batch;
    int *lists = nullptr;
    if (hipMalloc(&lists, kSrbdClasses * cap * sizeof(int)) != hipSuccess) return QLOCO_ERR_DEVICE;
    if (s.lists) {
      if (s.captured) {
        std::lock_guard<std::mutex> lp(g_srbd_pinned_mu);
        g_srbd_pinned.push_back(s.lists);  // a graph may still read the old lists
      } else {
        // every earlier use was enqueued on this stream
        if (hipStreamSynchronize(st) != hipSuccess) return QLOCO_ERR_DEVICE;
        (void)hipFree(s.lists);
      }
    }
    s.lists = lists;
    s.cap = cap;
  }
  if (capturing) s.captured = true;
  s.last_use = ++g_srbd_tick;
  *out = &s;
  return QLOCO_OK;
}

extern "C" int qloco_srbd_max_stance_vars(void) { return 3 * kBigLegs; }

// Which kernel family a call takes (qloco_srbd_route).  The wrench-space
// kernels build G^-1 from per-axis blocks: that needs every
// q_omega and q_v > 0 (G positive definite; any q_theta / q_p >= 0 -- the
// omega x / y pair is diagonalised with the yaw-rotated q_theta, so
// anisotropic omega weights stay on them) and feet constant over the
// horizon (the wrench map Bb is per instance).  They also need state
// weights of at most kLitMaxQ: their float32 push-through solve
// x = a - W0^-1 Vu' T Vu a cancels more digits as the wrench part of P grows
// against R at small rho, and with isaac_a1_mpc.yaml's weights (roll 8000,
// z 6020, v 2130) 1-2 % of N = 10 and 6-19 % of N = 11..16 instances stop
// converging at rho <= 3e-4 where float64 converges; T rounded from an exact
// float64 inverse does the same in emulation, so it is the form's precision,
// not the Gauss-Jordan's (tools/lit_weights_numerics.py).  The
// Go1 / gazebo / hardware sets (<= 420) match the float64 iteration counts.
// Other literal calls take the generic literal kernels (the 12N-variable
// KKT inverse), which converge on isaac's weights as float64 does.
constexpr float kLitMaxQ = 1000.0f;
static int srbd_route_of(const SrbdArgs &a) {
  if (!a.literal) return QLOCO_ROUTE_REDUCED;
  const bool lit_blocks = a.q2[6] > 0.0f && a.q2[7] > 0.0f && a.q2[8] > 0.0f && a.q2[9] > 0.0f &&
                          a.q2[10] > 0.0f && a.q2[11] > 0.0f;
  float qmax = 0.0f;
  for (int k = 0; k < 12; ++k) qmax = fmaxf(qmax, 0.5f * a.q2[k]);
  if (a.N <= kLitN2 && !a.feet_per_step && lit_blocks && qmax <= kLitMaxQ)
    return a.N <= kLitN ? QLOCO_ROUTE_LIT_ONE_WAVE : QLOCO_ROUTE_LIT_TWO_WAVE;
  return QLOCO_ROUTE_LIT_GENERIC;
}

extern "C" int qloco_srbd_route(const qloco_srbd_spec *spec) {
  if (!spec || spec->horizon < 1 || spec->horizon > kMaxN) return QLOCO_ERR_ARG;
  SrbdArgs a;
  memset(&a, 0, sizeof(a));
  a.N = spec->horizon;
  a.feet_per_step = spec->feet_per_step;
  a.literal = spec->literal_full_qp ? 1 : 0;
  for (int k = 0; k < 13; ++k) a.q2[k] = 2.0f * spec->q_weights[k];
  return srbd_route_of(a);
}

extern "C" int qloco_srbd_solve_ex(const qloco_srbd_spec *spec, int64_t batch, const float *x0,
                                   const float *x_ref, const float *feet,
                                   const uint8_t *contacts, float *u0, float *u,
                                   int32_t *status, int32_t *iters, int32_t *rho_updates,
                                   float *obj, float *warm, int32_t max_stance_legs,
                                   void *stream) {
  if (!spec || batch < 0) return QLOCO_ERR_ARG;
  if (spec->horizon < 1 || spec->horizon > kMaxN) return QLOCO_BAD_SIZE;
  if (batch == 0) return QLOCO_OK;
  if (!x0 || !x_ref || !feet || !contacts || !u0) return QLOCO_ERR_ARG;
  if (spec->warm_start < 0 || spec->warm_start > 2) return QLOCO_ERR_ARG;
  if (spec->warm_start && !warm) return QLOCO_ERR_ARG;
  if (spec->mass <= 0.0f || spec->dt <= 0.0f) return QLOCO_ERR_ARG;
  // OSQP polishing (off in OSQP's defaults and in the reference, which never
  // enables it, A1RobotControl.cpp:558-559) is not implemented: refuse rather
  // than return unpolished iterates as if polished
  if (spec->polish) return QLOCO_ERR_ARG;
  if (spec->literal_full_qp < 0 || spec->literal_full_qp > 1) return QLOCO_ERR_ARG;
  SrbdArgs a;
  memset(&a, 0, sizeof(a));
  a.N = spec->horizon;
  a.feet_per_step = spec->feet_per_step;
  a.contacts_per_step = spec->contacts_per_step;
  a.output_frame = spec->output_frame;
  a.dt = spec->dt;
  a.mass = spec->mass;
  for (int k = 0; k < 9; ++k) a.inertia[k] = spec->inertia[k];
  for (int k = 0; k < 13; ++k) a.q2[k] = 2.0f * spec->q_weights[k];
  for (int k = 0; k < 12; ++k) a.r2[k] = 2.0f * spec->r_weights[k];
  a.mu = spec->mu;
  a.fz_min = spec->fz_min;
  a.fz_max = spec->fz_max;
  a.rho = spec->rho;
  a.sigma = spec->sigma;
  a.alpha = spec->alpha;
  a.eps_abs = spec->eps_abs;
  a.eps_rel = spec->eps_rel;
  a.max_iter = spec->max_iter;
  a.check_termination = spec->check_termination;
  a.scaling = spec->scaling;
  a.adaptive_rho = spec->adaptive_rho;
  a.rho_interval = spec->adaptive_rho_interval;
  a.rho_tol = spec->adaptive_rho_tolerance;
  a.warm_start = spec->warm_start;
  a.literal = spec->literal_full_qp ? 1 : 0;
  a.batch = batch;
  a.x0 = x0;
  a.xref = x_ref;
  a.feet = feet;
  a.contacts = contacts;
  a.u0 = u0;
  a.u = u;
  a.obj = obj;
  a.warm = warm;
  a.status = status;
  a.iters = iters;
  a.rho_updates = rho_updates;
  // Kernel per instance class: <= 21 stance legs one-wave workgroups,
  // 22..42 two-wave workgroups, 43..80 the wide kernel (qloco_srbd_big.inc).
  // A batch that may hold several classes (the caller's maximum, or 4N when
  // unknown, says so) is first classified on the device (srbd_classify_kernel:
  // one compact instance list per class), then every class kernel walks only
  // its own list -- no workgroup is spent on another class's instance -- and
  // the classes run concurrently: class 0 on the caller's stream, classes 1
  // and 2 on the device's side streams between a fork and a join event, so
  // one class's tail overlaps another's bulk.  The top class the caller's
  // maximum admits takes every instance above the lower classes, so an
  // instance beyond a too-small maximum gets QLOCO_BAD_SIZE there.
  // the literal full QP has 4N "legs" (variable triples) in every instance
  const int legs = (a.literal || max_stance_legs <= 0) ? 4 * spec->horizon : max_stance_legs;
  hipStream_t st = (hipStream_t)stream;
  a.leg_lo = 0;
  a.leg_hi = 1 << 30;
  const bool ws = spec->warm_start != 0;
  const dim3 grid((unsigned)batch);
  auto launch = [&](int cls, hipStream_t s) {
    if (cls == 0) {
      if (a.N <= kShortN) {
        // short horizons: per-step tables sized for N <= 10 (9 KB of LDS) so
        // 16 one-wave workgroups share a CU -- four waves per SIMD
        if (ws)
          hipLaunchKernelGGL((srbd_admm_kernel<1, kShortWpe, true, kShortN>), grid, dim3(64), 0, s, a);
        else
          hipLaunchKernelGGL((srbd_admm_kernel<1, kShortWpe, false, kShortN>), grid, dim3(64), 0, s, a);
      } else if (batch <= kSmallBatch) {
        if (ws)
          hipLaunchKernelGGL((srbd_admm_kernel<1, kW1SmallWpe, true>), grid, dim3(64), 0, s, a);
        else
          hipLaunchKernelGGL((srbd_admm_kernel<1, kW1SmallWpe, false>), grid, dim3(64), 0, s, a);
      } else {
        if (ws)
          hipLaunchKernelGGL((srbd_admm_kernel<1, kW1Wpe, true>), grid, dim3(64), 0, s, a);
        else
          hipLaunchKernelGGL((srbd_admm_kernel<1, kW1Wpe, false>), grid, dim3(64), 0, s, a);
      }
    } else if (cls <= 4) {  // two-wave column buckets C2 = 3 / 6 / 9 / 15
      if (ws)  // srbd_class_of routes every warm two-wave instance to bucket 4
        hipLaunchKernelGGL((srbd_admm_kernel<2, kW2WarmWpe, true, kMaxN, 15>), grid, dim3(128), 0, s, a);
      else if (cls == 1)
        hipLaunchKernelGGL((srbd_admm_kernel<2, kW2Wpe, false, kMaxN, 3>), grid, dim3(128), 0, s, a);
      else if (cls == 2)
        hipLaunchKernelGGL((srbd_admm_kernel<2, kW2Wpe, false, kMaxN, 6>), grid, dim3(128), 0, s, a);
      else if (cls == 3)
        hipLaunchKernelGGL((srbd_admm_kernel<2, kW2Wpe, false, kMaxN, 9>), grid, dim3(128), 0, s, a);
      else
        hipLaunchKernelGGL((srbd_admm_kernel<2, kW2Wpe, false, kMaxN, 15>), grid, dim3(128), 0, s, a);
    } else {  // wide kernel half widths HC = 96 / 112 / 120
      if (ws)  // srbd_class_of routes every warm wide instance to class 7: one
               // warm instantiation at the full 128-column halves
        hipLaunchKernelGGL((srbd_admm_big_kernel<true, 128>), grid, dim3(kBigThreads), 0, s, a);
      else if (cls == 5)
        hipLaunchKernelGGL((srbd_admm_big_kernel<false, 96>), grid, dim3(kBigThreads), 0, s, a);
      else if (cls == 6)
        hipLaunchKernelGGL((srbd_admm_big_kernel<false, 112>), grid, dim3(kBigThreads), 0, s, a);
      else
        hipLaunchKernelGGL((srbd_admm_big_kernel<false, 120>), grid, dim3(kBigThreads), 0, s, a);
    }
  };
  const int top = srbd_class_of(legs, ws);
  if (srbd_route_of(a) <= QLOCO_ROUTE_LIT_TWO_WAVE) {
    // the literal QP at N <= 20 through the wrench space: one wave per
    // instance for N <= 10, two for 11..20 (qloco_srbd_lit.hip)
    const int rc = srbd_lit_launch(a, ws, st);
    if (rc != QLOCO_OK) return rc;
  } else if (top == 0 || a.literal) {
    // one class: every instance of the literal QP has 4N leg triples, so no
    // classification and no empty class launches
    launch(top, st);
  } else {
    std::unique_lock<std::mutex> lk(g_srbd_scratch_mu);
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    const bool capturing =
        hipStreamIsCapturing(st, &cst) == hipSuccess && cst != hipStreamCaptureStatusNone;
    SrbdScratch *sc = nullptr;
    SrbdScratch victim;
    // an evicted set is released after the lock is dropped, whatever the exit
    struct ReleaseAfterUnlock {
      std::unique_lock<std::mutex> &lk;
      SrbdScratch &v;
      ~ReleaseAfterUnlock() {
        if (lk.owns_lock()) lk.unlock();
        if (v.counts || v.lists) srbd_release(v);
      }
    } release_victim{lk, victim};
    const int rc = srbd_scratch(batch, st, capturing, &sc, &victim);
    if (rc != QLOCO_OK) return rc;
    QLOCO_HIP_CHECK(hipMemsetAsync(sc->counts, 0, 8 * sizeof(int), st), "class counters");
    hipLaunchKernelGGL(srbd_classify_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, st,
                       a, top, sc->lists, sc->cap, sc->counts);
    QLOCO_HIP_CHECK(hipGetLastError(), "srbd_classify_kernel launch");
    const bool fork = true;  // classes on the side streams (concurrent tails)
    if (fork) QLOCO_HIP_CHECK(hipEventRecord(sc->fork, st), "fork event");
    // class 0 on the caller's stream; two-wave buckets 1 / 3 on side stream
    // 0 and 2 / 4 on side stream 1 (a bucket's tail overlaps the next one's
    // bulk); the wide buckets in order on side stream 2
    bool waited[3] = {false, false, false};
    int last[3] = {-1, -1, -1};
    auto side_of = [](int c) { return c >= 5 ? 2 : ((c & 1) ? 0 : 1); };
    auto skip = [&](int c) {  // empty by construction (srbd_class_of)
      return ws && ((c >= 1 && c <= 3) || c == 5 || c == 6);
    };
    for (int c = 0; c <= top; ++c)
      if (c > 0 && !skip(c)) last[side_of(c)] = c;
    for (int c = 0; c <= top; ++c) {
      if (skip(c)) continue;
      a.list = sc->lists + (int64_t)c * sc->cap;
      a.count = sc->counts + c;
      a.leg_lo = 0;
      a.leg_hi = 1 << 30;
      const int sd = side_of(c);
      hipStream_t s = st;
      if (fork && c > 0) {
        s = sc->side[sd];
        if (!waited[sd]) QLOCO_HIP_CHECK(hipStreamWaitEvent(s, sc->fork, 0), "fork wait");
        waited[sd] = true;
      }
      launch(c, s);
      QLOCO_HIP_CHECK(hipGetLastError(), "srbd class kernel launch");
      if (fork && c > 0 && c == last[sd]) {
        QLOCO_HIP_CHECK(hipEventRecord(sc->join[sd], s), "join event");
        QLOCO_HIP_CHECK(hipStreamWaitEvent(st, sc->join[sd], 0), "join wait");
      }
    }
    // the set's last eager use (what a later release waits for)
    if (!capturing) {
      QLOCO_HIP_CHECK(hipEventRecord(sc->done, st), "scratch done event");
      sc->done_recorded = true;
    }
  }
  QLOCO_HIP_CHECK(hipGetLastError(), "srbd_admm_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_srbd_solve(const qloco_srbd_spec *spec, int64_t batch, const float *x0,
                                const float *x_ref, const float *feet, const uint8_t *contacts,
                                float *u0, float *u, int32_t *status, int32_t *iters, float *obj,
                                float *warm, void *stream) {
  return qloco_srbd_solve_ex(spec, batch, x0, x_ref, feet, contacts, u0, u, status, iters,
                             nullptr, obj, warm, 0, stream);
}
