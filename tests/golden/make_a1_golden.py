"""Generate tests/golden/a1_qp.npz: inputs and oracle outputs of the A1
single-step force QP (oracle/a1_qp.c restating A1RobotControl.cpp:383-450).
Data only (inputs, body-frame forces, iterations, status).
    python tests/golden/make_a1_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle_lib as O  # noqa: E402
from quadrupedal_loco_amd import a1qp  # noqa: E402

S, CT = a1qp.synth_states(20261016, 32)
F = np.zeros((32, 12))
it = np.zeros(32, np.int32)
st = np.zeros(32, np.int32)
for b in range(32):
    F[b], _, info = O.a1_compute_grf(S[b], CT[b])
    it[b], st[b] = info.iters, info.status
np.savez_compressed(os.path.join(HERE, "a1_qp.npz"), state=S, contacts=CT, forces=F, iters=it,
                    status=st)
print("wrote a1_qp.npz", it.min(), it.max(), np.unique(st))
