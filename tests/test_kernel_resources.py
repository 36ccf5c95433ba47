"""Register / scratch budget of every kernel in libqloco.so (CPU: reads the
gfx950 code objects' AMDGPU metadata, no GPU needed).

Guards the round-4 register plan: the one-wave headline
kernels run at four waves per SIMD (<= 128 VGPRs, <= 10 KB of LDS), every
kernel is spill-free except the listed ones, whose spill counts may not grow
(they sit outside the ADMM inner loops)."""
import os
import re
import shutil
import struct
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "quadrupedal_loco_amd", "lib", "libqloco.so")
READELF = shutil.which("llvm-readelf", path="/opt/rocm/lib/llvm/bin:/opt/rocm/llvm/bin") or shutil.which(
    "llvm-readelf")

# spilled VGPRs allowed (upper bounds, the round-4 build)
SPILL_BOUND = {
    "_ZN5qloco16srbd_admm_kernelILi1ELi4ELb1ELi10ELi16EEEvNS_8SrbdArgsE": 1,    # warm-start one-wave
    "_ZN5qloco16srbd_admm_kernelILi2ELi3ELb0ELi20ELi15EEEvNS_8SrbdArgsE": 33,   # C2 = 15 bucket
    "_ZN5qloco20srbd_admm_big_kernelILb1ELi128EEEvNS_8SrbdArgsE": 34,           # warm wide kernel
    "_ZN5qloco20srbd_admm_big_kernelILb0ELi120EEEvNS_8SrbdArgsE": 3,
}
# no scratch at all: the literal kernels keep their cross-phase scalars and
# per-slot vectors in LDS
NO_SCRATCH = [
    "_ZN5qloco15srbd_lit_kernelILb0EEEvNS_8SrbdArgsE",
    "_ZN5qloco15srbd_lit_kernelILb1EEEvNS_8SrbdArgsE",
    "_ZN5qloco16srbd_lit2_kernelILb0EEEvNS_8SrbdArgsE",
    "_ZN5qloco16srbd_lit2_kernelILb1EEEvNS_8SrbdArgsE",
    "_ZN5qloco16srbd_admm_kernelILi1ELi4ELb0ELi10ELi16EEEvNS_8SrbdArgsE",
]
# two waves per SIMD, 128-thread workgroups (the literal QP at N = 11..20: a
# 120-register row of S / T per lane)
TWO_WAVE = [
    "_ZN5qloco16srbd_lit2_kernelILb0EEEvNS_8SrbdArgsE",
    "_ZN5qloco16srbd_lit2_kernelILb1EEEvNS_8SrbdArgsE",
]
# four waves per SIMD: 128 VGPRs and 16 one-wave workgroups' LDS per CU
FOUR_WAVE = [
    "_ZN5qloco16srbd_admm_kernelILi1ELi4ELb0ELi10ELi16EEEvNS_8SrbdArgsE",
    "_ZN5qloco15srbd_lit_kernelILb0EEEvNS_8SrbdArgsE",
]


def _kernels():
    if not os.path.exists(LIB):
        pytest.skip("libqloco.so not built")
    if READELF is None:
        pytest.skip("llvm-readelf not available")
    data = open(LIB, "rb").read()
    out = []
    tmp = os.path.join(os.environ.get("TMPDIR", "/tmp"), "qloco_co_%d.o" % os.getpid())
    try:
        for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data):
            o = m.start()
            (n,) = struct.unpack_from("<Q", data, o + 24)
            p = o + 32
            for _ in range(n):
                off, size, tl = struct.unpack_from("<QQQ", data, p)
                p += 24
                triple = data[p:p + tl].decode()
                p += tl
                if "gfx950" not in triple or size == 0:
                    continue
                with open(tmp, "wb") as f:
                    f.write(data[o + off:o + off + size])
                notes = subprocess.run([READELF, "--notes", tmp], capture_output=True, text=True,
                                       check=True).stdout
                meta = yaml.safe_load(notes[notes.index("---"):notes.rindex("...")])
                out += meta["amdhsa.kernels"]
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return {k[".name"]: k for k in out}


@pytest.fixture(scope="module")
def kernels():
    return _kernels()


def test_every_kernel_is_gfx950_and_listed(kernels):
    assert len(kernels) >= 30
    for name in list(SPILL_BOUND) + FOUR_WAVE + TWO_WAVE + NO_SCRATCH:
        assert name in kernels, name


def test_spill_budget(kernels):
    over = []
    for name, k in kernels.items():
        bound = SPILL_BOUND.get(name, 0)
        if k[".vgpr_spill_count"] > bound:
            over.append((name, k[".vgpr_spill_count"], bound))
        assert not k.get(".uses_dynamic_stack", False), name
    assert not over, over


def test_headline_kernels_fit_four_waves_per_simd(kernels):
    for name in FOUR_WAVE:
        k = kernels[name]
        assert k[".vgpr_count"] + k[".agpr_count"] <= 128, (name, k[".vgpr_count"])
        assert k[".group_segment_fixed_size"] <= 10240, (name, k[".group_segment_fixed_size"])
    for name in NO_SCRATCH:
        assert kernels[name][".private_segment_fixed_size"] == 0, name


def test_two_wave_literal_kernel_budget(kernels):
    """The two-wave literal kernel: <= 256 registers (two waves
    per SIMD), LDS for four workgroups per CU, spill-free."""
    for name in TWO_WAVE:
        k = kernels[name]
        assert k[".vgpr_count"] + k[".agpr_count"] <= 256, (name, k[".vgpr_count"])
        assert k[".group_segment_fixed_size"] <= 40960, (name, k[".group_segment_fixed_size"])
        assert k[".vgpr_spill_count"] == 0 and k[".private_segment_fixed_size"] == 0, name


# the force QP: 8-lane groups (grouped launch) and 16-lane
# groups (ungrouped), both spill-free at two waves' register budget; the
# 8-robot block's LDS lets six blocks share a CU's 160 KB
FORCE_GW8 = "_ZN5qloco15force_qp_kernelILi8EEEvNS_9ForceArgsE"
FORCE_GW16 = "_ZN5qloco15force_qp_kernelILi16EEEvNS_9ForceArgsE"


def test_force_qp_kernel_budget(kernels):
    for name in (FORCE_GW8, FORCE_GW16):
        k = kernels[name]
        assert k[".vgpr_count"] + k[".agpr_count"] <= 256, (name, k[".vgpr_count"])
        assert k[".vgpr_spill_count"] == 0 and k[".private_segment_fixed_size"] == 0, name
    assert 6 * kernels[FORCE_GW8][".group_segment_fixed_size"] <= 160 * 1024
