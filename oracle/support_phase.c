/*
 * support_phase.c -- restatement of the slow planner's contact-phase flag
 * (mosek_nlp_kmp NLPClass, SURVEY.md §8f row 2 "NLP right_support logic"):
 * the schedule indices NLPClass::step_timing_opti_loop derives once its
 * step-timing SQP has updated _ts / _tx (NLPClass_sqp.cpp:1029-1039), and
 * the right_support branch of Foot_trajectory_solve_mod2 (:2076-2090,
 * :2187-2202, :2311-2313) that the NLP node publishes in /MPC/Gait[99]
 * (NLPRTControlClass.cpp:459, :544, :392) and servo.cpp:673 reads back.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned (the
 * reference needs ROS / Eigen); the integer outputs are compared bit for bit.
 *
 * Per robot, with dt = NLPClass _dt = 0.025 (NLPClass.h:32) and i = _t_int:
 *   bjxx = Indexfind(i * dt, xyz1) + 1                          (:1031-1032)
 *   bjx1 = Indexfind(_t_f(0), xyz1) + 1, _t_f(0) = (i + 1) * dt  (:1029, :1035-1036)
 *     Indexfind(g, 0): first j with g < _tx(j), minus 1 (:1105-1142),
 *     bounded at the 27 footsteps (the reference reads past the end)
 *   _td = 0.2 * _ts                                               (:1039)
 *   right_support (Foot_trajectory_solve_mod2):
 *     bjx1 >= 2 and i <= _t_end_footstep:
 *       bjx1 even -> 0 (left support), odd -> 1 (right support),
 *       then 2 (double support) when
 *       (i + 1 - round(_tx(bjx1 - 1) / dt)) * dt < _td(bjx1 - 1)
 *     otherwise 2.
 */
#include "qloco_oracle.h"

#include <math.h>

#define SP_NS 27
static const double SP_DT = 0.025;

static int sp_indexfind(const double *tx, double goal) {
  int j = 0;
  while (j < SP_NS && goal >= tx[j]) j++;
  return j - 1;
}

void qo_support_phase(int64_t n, const double *ts, const double *tx, const int32_t *t_int,
                      const int32_t *t_end_footstep, int32_t *bjxx, int32_t *bjx1,
                      int32_t *right_support) {
  for (int64_t r = 0; r < n; ++r) {
    const double *s = ts + SP_NS * r, *x = tx + SP_NS * r;
    const int i = t_int[r];
    const int bxx = sp_indexfind(x, i * SP_DT) + 1;
    const int b1 = sp_indexfind(x, (i + 1) * SP_DT) + 1;
    int rs = 2;
    if (b1 >= 2 && i <= t_end_footstep[r]) {
      const double td = 0.2 * s[b1 - 1];
      rs = (b1 % 2 == 0) ? 0 : 1;
      if ((i + 1 - round(x[b1 - 1] / SP_DT)) * SP_DT < td) rs = 2;
    }
    bjxx[r] = bxx;
    bjx1[r] = b1;
    right_support[r] = rs;
  }
}
