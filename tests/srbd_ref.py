"""Reference computations for the SRBD parity tests (test infrastructure).

Builds each instance's literal QP with the oracle (oracle/srbd.c), solves it
exactly (EiQuadProg restatement) and with the OSQP-algorithm ADMM
restatement, on the full 12N-variable problem and on the stance-only
reduction that the GPU kernel solves.
"""
import numpy as np

import oracle_lib as O


def stance_index(contacts, N):
    """Variable / row indices of stance (step, leg) pairs, ConvexMpc order."""
    idx, rows = [], []
    for k in range(N):
        for i in range(4):
            if contacts[4 * k + i]:
                idx += [12 * k + 3 * i + j for j in range(3)]
                rows += [20 * k + 5 * i + j for j in range(5)]
    return np.array(idx, dtype=np.int64), np.array(rows, dtype=np.int64)


class Instance:
    def __init__(self, spec, x0, xr, ft, ct, feet_per_step=0):
        self.N = N = spec.N
        self.ct = np.asarray(ct, np.uint8)
        self.H, self.g, self.lb, self.ub = O.build_instance(spec, x0, xr, ft, ct,
                                                            contacts_per_step=1,
                                                            feet_per_step=feet_per_step)
        self.A = O.constraints(spec)
        self.idx, self.rows = stance_index(self.ct, N)

    def obj(self, u):
        u = np.asarray(u, np.float64)
        return 0.5 * u @ self.H @ u + self.g @ u

    def exact(self):
        x, st, it = O.exact_solve(self.H, self.g, self.A, self.lb, self.ub)
        return x, st, it

    def admm_full(self, **kw):
        x, y, info = O.admm_solve(self.H, self.g, self.A, self.lb, self.ub,
                                  O.admm_settings(**kw))
        return x, info

    def admm_reduced(self, **kw):
        i, r = self.idx, self.rows
        H = self.H[np.ix_(i, i)]
        A = self.A[np.ix_(r, i)]
        xr, y, info = O.admm_solve(H, self.g[i], A, self.lb[r], self.ub[r], O.admm_settings(**kw))
        x = np.zeros(12 * self.N)
        x[i] = xr
        return x, info

    def violation(self, u):
        Au = self.A @ np.asarray(u, np.float64)
        return max(0.0, float(np.max(self.lb - Au)), float(np.max(Au - self.ub)))
