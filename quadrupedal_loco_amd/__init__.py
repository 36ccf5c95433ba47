"""quadrupedal_loco_amd -- MI355X-native batched convex-MPC solver.

Drop-in for the QP hot path of jtdingx/quadrupedal_loco (rt_mpc_qp body MPC,
go1_rt_control force QP, ConvexMpc SRBD MPC); see DESIGN.md.  The compute
runs in hand-written gfx950 HIP kernels behind the C ABI of include/qloco.h.
"""
from ._lib import QlocoError, lib, missing_symbols  # noqa: F401

__version__ = "0.1.0"
