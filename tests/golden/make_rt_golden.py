"""Generate tests/golden/rt_tick.npz: the rt_mpc_qp node tick restatement
(oracle/rt_tick.c) driven by quadrupedal_loco_amd.rt.synth_messages.

Saved: the input messages and the /rtMPC/traj, /rt2nrt/state and schedule
integers at a spread of ticks covering start-up, interpolation, swing,
step-period rewrites and the post-schedule stop branch.  Run from the repo
root:  python tests/golden/make_rt_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_lib as O  # noqa: E402
from quadrupedal_loco_amd.rt import synth_messages  # noqa: E402

SEED, B, T = 20261017, 8, 1900
SAVE = sorted(set([0, 1, 2, 3, 5, 50, 101, 102, 103, 150, 200, 250, 333, 500, 777, 1000, 1234,
                   1500, 1650, 1700, 1750, 1800, 1850, 1899]))


def main():
    orc = O.RtOracle(B)
    keep = {k: [] for k in ("gait", "ctrl", "traj", "nrt", "gen", "sched")}
    for t in range(T):
        gait, ctrl = synth_messages(SEED, B, t)
        traj, nrt, gen, sched = orc.tick(gait, ctrl)
        if t in SAVE:
            for k, v in zip(keep, (gait, ctrl, traj, nrt, gen, sched)):
                keep[k].append(v.copy())
    out = os.path.join(ROOT, "tests", "golden", "rt_tick.npz")
    np.savez_compressed(out, seed=SEED, batch=B, ticks=T, ticks_saved=np.array(SAVE),
                        **{k: np.stack(v) for k, v in keep.items()})
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
