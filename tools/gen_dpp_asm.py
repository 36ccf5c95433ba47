#!/usr/bin/env python3
"""Generate quadrupedal_loco_amd/csrc/qloco_dpp.inc: inline-asm blocks of
v_fmac_f32_dpp ... row_newbcast:j used by the SRBD kernel's K^-1 matvec and
Gauss-Jordan update (64 columns per block).

row_newbcast:j (DPP, gfx90a+) hands every lane the value lane j of its own
16-lane row holds.  Each lane loads one 16-byte chunk of the broadcast
vector (lane l: elements 4(l%16)..4(l%16)+3, one ds_read_b128 per wave
instead of sixteen), and the DPP operand of the FMA fans it out.  One
`s_nop 4` at the head of each block covers the VALU-write -> DPP-read and
EXEC-write -> DPP hazards for the source registers.

    python tools/gen_dpp_asm.py   # rewrites the .inc (checked in)
"""
import os

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "quadrupedal_loco_amd", "csrc", "qloco_dpp.inc")


def dpp(dst, src, other, j):
    return "v_fmac_f32_dpp %%%d, %%%d, %%%d row_newbcast:%d row_mask:0xf bank_mask:0xf" % (
        dst, src, other, j)


def matvec(acc, nch=16):
    # outputs A0..A3 = %0..%3, inputs R.x..R.w = %4..%7, KK[B+c] = %8+c.  Without
    # acc the first group is a v_mul (no accumulator zeroing).  R comes straight
    # from a ds_read (no VALU write); s_nop 1 covers a compiler-inserted copy.
    body = ["s_nop 1"]
    for j in range(nch):
        for e in range(4):
            if j == 0 and not acc:
                body.append("v_mul_f32_dpp %%%d, %%%d, %%%d row_newbcast:0 row_mask:0xf bank_mask:0xf"
                            % (e, 4 + e, 8 + e))
            else:
                body.append(dpp(e, 4 + e, 8 + 4 * j + e, j))
    outs = ", ".join(('"+v"(A%d)' if acc else '"=&v"(A%d)') % e for e in range(4))
    ins = ", ".join(['"v"((R).x)', '"v"((R).y)', '"v"((R).z)', '"v"((R).w)'] +
                    ['"v"((KK)[(B) + %d])' % c for c in range(4 * nch)])
    name = ("QL_DPP_MATVEC%d_ACC" if acc else "QL_DPP_MATVEC%d") % (4 * nch)
    what = "+=" if acc else "="
    return ("// A_e %s sum_j KK[B + 4j + e] * R_e(lane j of the row)\n" % what +
            "#define " + name + "(A0, A1, A2, A3, R, KK, B) \\\n  asm(\"" +
            "\\n\\t\" \\\n      \"".join(body) + "\" \\\n      : " + outs + " \\\n      : " + ins + ")\n")


def gj(nch=16):
    # outputs KK[B+c] = %c (c < 4 nch), inputs R.x..R.w = %nc..%nc+3, NG = %nc+4
    nc = 4 * nch
    body = ["s_nop 4"] + [dpp(4 * j + e, nc + e, nc + 4, j) for j in range(nch) for e in range(4)]
    outs = ", ".join('"+v"((KK)[(B) + %d])' % c for c in range(nc))
    ins = '"v"((R).x), "v"((R).y), "v"((R).z), "v"((R).w), "v"(NG)'
    return ("// KK[B + 4j + e] += R_e(lane j of the row) * NG, columns < %d\n" % nc +
            "#define QL_DPP_GJ%d(KK, B, R, NG) \\\n  asm(\"" % nc +
            "\\n\\t\" \\\n      \"".join(body) + "\" \\\n      : " + outs + " \\\n      : " + ins + ")\n")


def mul(nch=16):
    # in/out KK[B+c] = %c (c < 4 nch), inputs R = %nc..%nc+3: KK[B+4j+e] *= R_e(lane j)
    nc = 4 * nch
    body = ["s_nop 4"] + ["v_mul_f32_dpp %%%d, %%%d, %%%d row_newbcast:%d row_mask:0xf bank_mask:0xf"
                          % (4 * j + e, nc + e, 4 * j + e, j) for j in range(nch) for e in range(4)]
    outs = ", ".join('"+v"((KK)[(B) + %d])' % c for c in range(nc))
    ins = '"v"((R).x), "v"((R).y), "v"((R).z), "v"((R).w)'
    return ("// KK[B + 4j + e] *= R_e(lane j of the row), columns < %d\n" % nc +
            "#define QL_DPP_MUL%d(KK, B, R) \\\n  asm(\"" % nc +
            "\\n\\t\" \\\n      \"".join(body) + "\" \\\n      : " + outs + " \\\n      : " + ins + ")\n")


def absmax(nch=16):
    # outputs A0..A3 = %0..%3, temps T0..T3 = %4..%7 (early clobber),
    # inputs R = %8..%11, KK[B+c] = %12+c:  A_e = max(A_e, R_e(lane j) * |KK[B+4j+e]|)
    # two products per v_max3: 64 DPP multiplies + 32 max3 per 64 columns;
    # accumulators A0/A1 take the even / odd chunk halves, A2/A3 the next j
    body = ["s_nop 4"]
    for j in range(nch):
        for e in range(4):
            body.append("v_mul_f32_dpp %%%d, %%%d, |%%%d| row_newbcast:%d row_mask:0xf bank_mask:0xf"
                        % (4 + e, 8 + e, 12 + 4 * j + e, j))
        a0, a1 = (0, 1) if j % 2 == 0 else (2, 3)
        body.append("v_max3_f32 %%%d, %%%d, %%4, %%5" % (a0, a0))
        body.append("v_max3_f32 %%%d, %%%d, %%6, %%7" % (a1, a1))
    outs = ", ".join(['"+v"(A%d)' % e for e in range(4)] + ['"=&v"(T%d)' % e for e in range(4)])
    ins = ", ".join(['"v"((R).x)', '"v"((R).y)', '"v"((R).z)', '"v"((R).w)'] +
                    ['"v"((KK)[(B) + %d])' % c for c in range(4 * nch)])
    return ("// A_e = max(A_e, R_e(lane j of the row) * |KK[B + 4j + e]|); T0..T3 scratch\n"
            "#define QL_DPP_ABSMAX%d(A0, A1, A2, A3, T0, T1, T2, T3, R, KK, B) \\\n  asm(\"" % (4 * nch) +
            "\\n\\t\" \\\n      \"".join(body) + "\" \\\n      : " + outs + " \\\n      : " + ins + ")\n")


def matvec2(nch=16):
    # two accumulators (A0: components x,z; A1: y,w): outputs %0,%1, R = %2..%5, KK = %6+c
    body = ["s_nop 1"]
    for j in range(nch):
        for e in range(4):
            a = e % 2
            if j == 0 and e < 2:
                body.append("v_mul_f32_dpp %%%d, %%%d, %%%d row_newbcast:0 row_mask:0xf bank_mask:0xf"
                            % (a, 2 + e, 6 + e))
            else:
                body.append(dpp(a, 2 + e, 6 + 4 * j + e, j))
    outs = '"=&v"(A0), "=&v"(A1)'
    ins = ", ".join(['"v"((R).x)', '"v"((R).y)', '"v"((R).z)', '"v"((R).w)'] +
                    ['"v"((KK)[(B) + %d])' % c for c in range(4 * nch)])
    return ("// A0 + A1 = sum_j,e KK[B + 4j + e] * R_e(lane j of the row), two accumulators\n"
            "#define QL_DPP_MATVEC%d_2(A0, A1, R, KK, B) \\\n  asm(\"" % (4 * nch) +
            "\\n\\t\" \\\n      \"".join(body) + "\" \\\n      : " + outs + " \\\n      : " + ins + ")\n")


if __name__ == "__main__":
    with open(OUT, "w") as f:
        f.write("// Generated by tools/gen_dpp_asm.py -- do not edit.\n#pragma once\n\n")
        f.write(matvec(False) + "\n" + matvec(True) + "\n" + gj() + "\n" + mul() + "\n" +
                absmax() + "\n" + matvec2() + "\n" +
                # 60-column forms: n <= 60 (every N = 10 trot / pace instance) --
                # columns 60..63 are identity padding, their updates are zero
                gj(15) + "\n" + mul(15) + "\n" + absmax(15) + "\n" + matvec2(15) + "\n" +
                # W = 2 second-half forms (columns 64.. of the row): 60 and 36 columns
                matvec(True, 15) + "\n" + matvec(True, 9) + "\n" + gj(9) + "\n" + mul(9) + "\n" +
                absmax(9) + "\n" +
                # four-chain 60-column form (W = 1, QLOCO_MATVEC4)
                matvec(False, 15) + "\n" +
                # W = 2 second-half forms for the narrow buckets (<= 12 / <= 24
                # columns: 22-25 / 26-29 stance legs, the mixed schedules)
                matvec(True, 3) + "\n" + matvec(True, 6) + "\n" + gj(3) + "\n" + gj(6) + "\n" +
                mul(3) + "\n" + mul(6) + "\n" + absmax(3) + "\n" + absmax(6))
    print(OUT)
