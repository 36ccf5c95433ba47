"""Generate tests/golden/kin_ref.npz: Go1 leg kinematics vectors computed with
the REFERENCE's own arithmetic.

Kinematics.cpp cannot be compiled as a unit here (it includes ros/ros.h and
the unitree message headers, absent from the image).  Its computing part is
four blocks of plain expressions in q / body_P / body_R and the leg constants,
so this script reads them out of
/root/reference/unitree_ros/go1_rt_control/src/kinematics/Kinematics.cpp at
generation time, places them in a throwaway C harness in a temporary
directory, and evaluates them with gcc (-O2 -ffp-contract=off, x86-64 double).
Nothing of the reference is stored in the repository: the committed fixture
holds only inputs and outputs.  The Newton loops of Inverse_kinematics(_g)
(:233-304) are restated around the extracted FK expressions; Eigen's 3x3
inverse is restated with its cofactor order.

    python tests/golden/make_kin_golden.py     # needs /root/reference + gcc
"""
import os
import re
import subprocess
import tempfile

import numpy as np

REF = "/root/reference/unitree_ros/go1_rt_control/src/kinematics/Kinematics.cpp"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kin_ref.npz")


def _block(src, start):
    i = src.index(start)
    return src[i:src.index("return pos_feet;", i)]


def _exprs(block):
    feet = block[block.index("pos_feet <<") + len("pos_feet <<"):]
    feet = feet[:feet.index(";")]
    pos = [p.strip() for p in re.split(r",\s*\n", feet)]
    assert len(pos) == 3
    jac = dict(re.findall(r"Jacobian_kin\((\d,\d)\)\s*=\s*(.*?);", block, re.S))
    assert len(jac) == 9
    return pos, jac


def _harness(local, glob):
    pl, jl = local
    pg, jg = glob
    body = ["#include <math.h>", "#include <stdio.h>", "#include <stdlib.h>", "",
            "static void consts(int f, double *ox, double *oy, double *ty, double *tl, double *cl) {",
            "  *ox = (f == 0 || f == 1) ? 0.1881 : -0.1881;",
            "  *oy = (f == 0 || f == 2) ? -0.04675 : 0.04675;",
            "  *ty = (f == 0 || f == 2) ? -0.08 : 0.08;",
            "  *tl = -0.213; *cl = -0.213;", "}", ""]
    for name, (pos, jac), glob_args in (("fk_l", (pl, jl), False), ("fk_g", (pg, jg), True)):
        sig = "const double *P, const double *E, " if glob_args else ""
        body.append("static void %s(%sconst double *q, int f, double *pos, double *J) {" % (name, sig))
        body.append("  double leg_offset_x, leg_offset_y, thigh_y, thigh_length, calf_length;")
        body.append("  consts(f, &leg_offset_x, &leg_offset_y, &thigh_y, &thigh_length, &calf_length);")
        body.append("  double q_hip = q[0], q_thigh = q[1], q_calf = q[2];")
        if glob_args:
            body.append("  double body_px = P[0], body_py = P[1], body_pz = P[2];")
            body.append("  double body_r = E[0], body_p = E[1], body_y = E[2];")
        for r in range(3):
            body.append("  pos[%d] = %s;" % (r, pos[r]))
        for key, val in jac.items():
            r, c = map(int, key.split(","))
            body.append("  J[%d] = %s;" % (3 * c + r, val))
        body.append("}")
    body += [
        "static double cof(const double *A, int i, int j) {",
        "  int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;",
        "  return A[3 * j1 + i1] * A[3 * j2 + i2] - A[3 * j2 + i1] * A[3 * j1 + i2];", "}",
        "static void inv3(const double *A, double *Ai) {",
        "  double c0 = cof(A, 0, 0), c1 = cof(A, 1, 0), c2 = cof(A, 2, 0);",
        "  double invdet = 1.0 / (c0 * A[0] + c1 * A[1] + c2 * A[2]);",
        "  Ai[0] = c0 * invdet; Ai[3] = c1 * invdet; Ai[6] = c2 * invdet;",
        "  for (int r = 1; r < 3; r++) for (int c = 0; c < 3; c++) Ai[3 * c + r] = cof(A, c, r) * invdet;", "}",
        # IK loop, Kinematics.cpp:237-263 / :274-299
        "static int ik(int g, const double *P, const double *E, const double *pd, const double *qi, int f,",
        "              double *q, double *pos, double *J) {",
        "  double Ji[9], dp[3], da[3];",
        "  if (g) fk_g(P, E, qi, f, pos, J); else fk_l(qi, f, pos, J);",
        "  for (int r = 0; r < 3; r++) q[r] = qi[r];",
        "  int n = 0;",
        "  for (int j = 0; j < (g ? 15 : 10); j++) {",
        "    for (int r = 0; r < 3; r++) dp[r] = pd[r] - pos[r];",
        "    inv3(J, Ji);",
        "    for (int r = 0; r < 3; r++) da[r] = (0.5 * Ji[r]) * dp[0] + (0.5 * Ji[3 + r]) * dp[1] + (0.5 * Ji[6 + r]) * dp[2];",
        "    int stop;",
        "    if (g) stop = fabs(pow(dp[0], 2) + pow(dp[1], 2) + pow(dp[2], 2)) <= 0.000001;",
        "    else { double m = da[0]; if (da[1] > m) m = da[1]; if (da[2] > m) m = da[2]; stop = m < 0.0001; }",
        "    if (stop) break;",
        "    for (int r = 0; r < 3; r++) q[r] += da[r];",
        "    n++;",
        "    if (g) fk_g(P, E, q, f, pos, J); else fk_l(q, f, pos, J);",
        "  }",
        "  return n;", "}",
        # driver: stdin rows "mode f q0 q1 q2 P0 P1 P2 E0 E1 E2 d0 d1 d2" -> stdout
        "int main(void) {",
        "  int mode, f; double q[3], P[3], E[3], d[3], pos[3], J[9], qo[3];",
        "  while (scanf(\"%d %d %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf\", &mode, &f, q, q + 1, q + 2,",
        "               P, P + 1, P + 2, E, E + 1, E + 2, d, d + 1, d + 2) == 14) {",
        "    int n = 0;",
        "    if (mode == 0) { fk_l(q, f, pos, J); qo[0] = q[0]; qo[1] = q[1]; qo[2] = q[2]; }",
        "    else if (mode == 1) { fk_g(P, E, q, f, pos, J); qo[0] = q[0]; qo[1] = q[1]; qo[2] = q[2]; }",
        "    else n = ik(mode == 3, P, E, d, q, f, qo, pos, J);",
        "    printf(\"%d\", n);",
        "    for (int r = 0; r < 3; r++) printf(\" %a\", qo[r]);",
        "    for (int r = 0; r < 3; r++) printf(\" %a\", pos[r]);",
        "    for (int r = 0; r < 9; r++) printf(\" %a\", J[r]);",
        "    printf(\"\\n\");",
        "  }",
        "  return 0;", "}"]
    return "\n".join(body) + "\n"


def main():
    src = open(REF).read()
    local = _exprs(_block(src, "Eigen::Matrix<double, 3,1> Kinematicclass::Forward_kinematics("))
    glob = _exprs(_block(src, "Eigen::Matrix<double, 3,1> Kinematicclass::Forward_kinematics_g("))
    rng = np.random.default_rng(20261015)
    rows = []
    # mode 0/1: FK local / global; 2/3: IK local / global
    home = np.array([0.0, 0.87, -1.5])
    for f in range(4):  # known answer: homing pose (SURVEY.md §8d nominal feet)
        rows.append((0, f, home, np.zeros(3), np.zeros(3), np.zeros(3)))
    for k in range(400):
        f = k % 4
        q = np.array([rng.uniform(-0.8, 0.8), rng.uniform(-0.5, 2.5), rng.uniform(-2.7, -0.9)])
        P = np.array([rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(0.25, 0.35)])
        E = np.array([rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3), rng.uniform(-np.pi, np.pi)])
        rows.append((k % 2, f, q, P, E, np.zeros(3)))
    # IK targets: FK of a nearby pose, started from the homing pose / a perturbation
    for k in range(400):
        f = k % 4
        g = k % 2
        qt = home + np.array([rng.uniform(-0.3, 0.3), rng.uniform(-0.4, 0.4), rng.uniform(-0.4, 0.4)])
        P = np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(0.28, 0.33)])
        E = np.array([rng.uniform(-0.2, 0.2), rng.uniform(-0.2, 0.2), rng.uniform(-np.pi, np.pi)])
        rows.append((4 + g, f, qt, P, E, None))  # placeholder: target from FK below
        qi = qt + rng.uniform(-0.15, 0.15, 3) if k % 3 else home.copy()
        rows[-1] = (4 + g, f, qi, P, E, qt)
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "h.c")
        exe = os.path.join(td, "h")
        open(c, "w").write(_harness(local, glob))
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", c, "-lm", "-o", exe], check=True)

        def run(lines):
            out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True,
                                 text=True, check=True).stdout.split("\n")
            res = []
            for ln in out:
                if ln.strip():
                    tok = ln.split()
                    res.append((int(tok[0]), [float.fromhex(x) for x in tok[1:]]))
            return res

        def fmt(mode, f, q, P, E, d):
            return " ".join([str(mode), str(f)] + ["%r" % float(v) for v in (*q, *P, *E, *d)])

        # targets for the IK rows (reference FK of qt)
        tgt_lines = []
        for mode, f, q, P, E, qt in rows:
            if mode >= 4:
                tgt_lines.append(fmt(mode - 4, f, qt, P, E, np.zeros(3)))
        tgts = [np.array(r[1][3:6]) for r in run(tgt_lines)]
        lines, it = [], iter(tgts)
        final = []
        for mode, f, q, P, E, d in rows:
            if mode >= 4:
                d = next(it)
                mode = 2 + (mode - 4)
            final.append((mode, f, q, P, E, d))
            lines.append(fmt(mode, f, q, P, E, d))
        res = run(lines)
    mode = np.array([r[0] for r in final], np.int32)
    leg = np.array([r[1] for r in final], np.int32)
    q_in = np.array([r[2] for r in final])
    body_p = np.array([r[3] for r in final])
    body_r = np.array([r[4] for r in final])
    pos_des = np.array([r[5] for r in final])
    updates = np.array([r[0] for r in res], np.int32)
    vals = np.array([r[1] for r in res])
    np.savez(OUT, mode=mode, leg=leg, q_in=q_in, body_p=body_p, body_r=body_r, pos_des=pos_des,
             q_out=vals[:, 0:3], pos=vals[:, 3:6], jac=vals[:, 6:15], updates=updates)
    print(OUT, len(final), "rows; ik updates histogram",
          np.bincount(updates[mode >= 2], minlength=16).tolist())


if __name__ == "__main__":
    main()
