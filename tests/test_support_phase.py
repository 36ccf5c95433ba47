"""Slow planner's contact-phase flag ("NLP right_support
logic"): oracle/support_phase.c against an independent per-robot transcription
of NLPClass_sqp.cpp:1029-1039 / :1105-1142 / Foot_trajectory_solve_mod2's
right_support branches (:2076-2090, :2187-2202, :2311-2313), and the HIP kernel
(qloco_support_phase) against the oracle, bit for bit.  Parity unpinned: the
reference needs ROS / Eigen and holds no fixtures for this path."""
import math

import numpy as np
import pytest

import oracle_lib as O
from quadrupedal_loco_amd.rt import synth_schedules

DT = 0.025


def _cround(x):
    """C round() (half away from zero) for x >= 0; x - floor(x) is exact"""
    f = math.floor(x)
    return f + 1.0 if x - f >= 0.5 else float(f)


def _transcribed(ts, tx, i, t_end):
    """per robot, as NLPClass writes it (Indexfind with xyz1; _td = 0.2 _ts)"""
    def indexfind(goal):
        j = 0
        while j < 27 and goal >= tx[j]:
            j += 1
        return j - 1
    bjxx = indexfind(i * DT) + 1
    t_f0 = (i + 1) * DT
    bjx1 = indexfind(t_f0) + 1
    td = [0.2 * v for v in ts]
    if bjx1 >= 2 and i <= t_end:
        rs = 0 if bjx1 % 2 == 0 else 1
        if (i + 1 - _cround(tx[bjx1 - 1] / DT)) * DT < td[bjx1 - 1]:
            rs = 2
    else:
        rs = 2
    return bjxx, bjx1, rs


def _edge_cases():
    """robots on the exact grid boundaries, before the second step, past
    t_end_footstep, and at the last step"""
    ts0, tx0, _, _ = synth_schedules(7, 1)
    rows_ts, rows_tx, ti, te = [], [], [], []
    t_end = int(np.round((tx0[0, 26] - 1.4) / DT))
    for j in range(27):
        g = int(math.floor(tx0[0, j] / DT))
        for i in (g - 1, g, g + 1, g + 2):
            if i < 0:
                continue
            rows_ts.append(ts0[0])
            rows_tx.append(tx0[0])
            ti.append(i)
            te.append(t_end if j % 3 else i - 1)
    for i in (0, 1, 27, 28):  # bjx1 < 2 on the first step
        rows_ts.append(ts0[0])
        rows_tx.append(tx0[0])
        ti.append(i)
        te.append(t_end)
    big = 10 ** 6  # past every step: the scan stops at 27
    rows_ts.append(ts0[0])
    rows_tx.append(tx0[0])
    ti.append(big)
    te.append(big)
    return (np.array(rows_ts), np.array(rows_tx), np.array(ti, np.int32),
            np.array(te, np.int32))


def test_oracle_matches_transcription():
    for ts, tx, ti, te in (synth_schedules(20261018, 3000), _edge_cases()):
        bxx, b1, rs = O.support_phase(ts, tx, ti, te)
        for r in range(len(ti)):
            assert (bxx[r], b1[r], rs[r]) == _transcribed(ts[r], tx[r], int(ti[r]), int(te[r])), r
    ts, tx, ti, te = synth_schedules(20261018, 3000)
    _, b1, rs = O.support_phase(ts, tx, ti, te)
    counts = np.bincount(rs, minlength=3)
    assert (counts > 100).all(), counts  # every phase is exercised
    assert (b1 >= 2).mean() > 0.9


def test_reference_semantics():
    """left support on even steps, right on odd, double support for the
    first _td = 0.2 _ts of every step (NLPClass_sqp.cpp:2079-2093)"""
    ts, tx, ti, te = synth_schedules(5, 2000)
    te[:] = 10 ** 6
    _, b1, rs = O.support_phase(ts, tx, ti, te)
    r = np.arange(len(ti))
    in_dsp = (ti + 1 - np.round(tx[r, b1 - 1] / DT)) * DT < 0.2 * ts[r, b1 - 1]
    ok = b1 >= 2
    assert ((rs == 2) == (in_dsp | ~ok)).all()
    assert (rs[ok & ~in_dsp] == (b1[ok & ~in_dsp] % 2)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 63, 65, 4096])
def test_gpu_matches_oracle(B):
    import torch
    from quadrupedal_loco_amd.rt import support_phase
    dev = torch.device("cuda:0")
    ts, tx, ti, te = synth_schedules(20261019 + B, B)
    got = support_phase(*[torch.from_numpy(a).to(dev) for a in (ts, tx, ti, te)])
    want = O.support_phase(ts, tx, ti, te)
    for g, w in zip(got, want):
        assert np.array_equal(g.cpu().numpy(), w)


@pytest.mark.gpu
def test_gpu_edge_cases_and_full_size():
    import torch
    from quadrupedal_loco_amd.rt import support_phase
    dev = torch.device("cuda:0")
    for arrays in (_edge_cases(), synth_schedules(3, 1 << 20)):
        got = support_phase(*[torch.from_numpy(a).to(dev) for a in arrays])
        want = O.support_phase(*arrays)
        for g, w in zip(got, want):
            assert np.array_equal(g.cpu().numpy(), w)


@pytest.mark.gpu
def test_gpu_bad_args():
    import torch
    from quadrupedal_loco_amd import _lib
    from quadrupedal_loco_amd.rt import support_phase
    dev = torch.device("cuda:0")
    L = _lib.lib()
    assert L.qloco_support_phase(-1, None, None, None, None, None, None, None, None) != 0
    assert L.qloco_support_phase(0, None, None, None, None, None, None, None, None) == 0
    assert L.qloco_support_phase(4, None, None, None, None, None, None, None, None) != 0
    ts, tx, ti, te = [torch.from_numpy(a).to(dev) for a in synth_schedules(1, 8)]
    with pytest.raises(ValueError):
        support_phase(ts.float(), tx, ti, te)
    with pytest.raises(ValueError):
        support_phase(ts[:, :26].contiguous(), tx, ti, te)
