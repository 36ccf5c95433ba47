"""GPU test of the C++ host shim (include/qloco.hpp, libqloco_host.so).

Runs tests/cpp/test_host (built by __graft_entry__.build() /
quadrupedal_loco_amd.build.build_host_test), which drives the shim classes
with the reference's call sequences and checks them against the oracle; see
the header of tests/cpp/test_host.cpp for the cases and tolerances.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_build", "test_host")


def test_cpp_shim_against_oracle():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        from quadrupedal_loco_amd import build as qb
        qb.build()
        qb.build_host_test(os.path.join(ROOT, "oracle", "_build", "libqloco_oracle.so"))
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
