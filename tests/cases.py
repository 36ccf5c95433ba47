"""Shared synthetic inputs for parity tests and golden generation."""
import numpy as np

import oracle_lib as O


def force_inputs(rng, B):
    homing = np.array([[0.150786, -0.12675, 0.0], [0.150786, 0.12675, 0.0],
                       [-0.225414, -0.12675, 0.0], [-0.225414, 0.12675, 0.0]])
    base = np.array([0.0, 0.0, 0.309458]) + rng.uniform(-0.02, 0.02, (B, 3))
    feet = homing[None] + rng.uniform(-0.03, 0.03, (B, 4, 3))
    feet[..., 2] = rng.uniform(-0.005, 0.005, (B, 4))
    acc = rng.normal(0, 0.5, (B, 3))
    mass = 12.0
    I = O.GO1_INERTIA
    F_sum = np.concatenate([mass * acc[:, :2], (mass * 9.8 + mass * acc[:, 2:3]),
                            acc @ I.T], axis=1)
    mode = rng.choice([101, 102, 103], B).astype(np.int32)
    rs = rng.integers(0, 3, B).astype(np.int32)
    rfoot = (feet[:, 0] + feet[:, 3]) / 2
    lfoot = (feet[:, 1] + feet[:, 2]) / 2
    y = np.where(mode == 101, 0.75, np.where(mode == 102, 0.0, 0.11))
    return dict(com_des=base, leg_des=feet.reshape(B, 12), F_force_des=F_sum,
                rfoot_des=rfoot, lfoot_des=lfoot, base_p=base, feet_p=feet.reshape(B, 12),
                FT_total_des=F_sum, mode=mode, right_support=rs, y_coef=y)
