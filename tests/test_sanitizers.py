"""Sanitizer runs of the host-side code (CPU only).

* The oracle (every restatement, including the paths that emulate reference
  undefined behaviour: EiQuadProg's `qq` search and skipped zero CE columns,
  Indexfind past the 27-step schedule, the body QP's inert CI columns) under
  AddressSanitizer + UndefinedBehaviorSanitizer: `make -C oracle asan` builds
  oracle/_build_asan/asan_check, driven with a long rt walk and force-QP
  inputs written here.
* The Python CPU tests of the oracle paths with the UBSan build of the oracle
  library loaded in place of the plain one (QLOCO_ORACLE_UBSAN=1).
* The C++ shim (host/qloco_host.cpp) under ASan + UBSan on this GPU-less
  host: constructor checks, the no-GPU refusal, C ABI argument validation.
GPU code is not sanitized (no GPU ASan / xnack on this pool)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


def _env(**extra):
    e = dict(os.environ)
    e.update(SAN_ENV)
    e.update(extra)
    return e


def test_oracle_under_asan_ubsan(tmp_path):
    import oracle_lib as O
    from cases import force_inputs
    from quadrupedal_loco_amd.rt import synth_messages
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True)
    T, B = 1200, 8
    with open(tmp_path / "rt_msgs.bin", "wb") as f:
        np.array([T, B], np.int32).tofile(f)
        for t in range(T):
            g, c = synth_messages(20261016, B, t)
            np.ascontiguousarray(g, np.float64).tofile(f)
            np.ascontiguousarray(c, np.float64).tofile(f)
    d = force_inputs(np.random.default_rng(3), 64)
    with open(tmp_path / "force.bin", "wb") as f:
        np.array([64], np.int32).tofile(f)
        for b in range(64):
            rec = np.zeros(52)
            rec[0:3], rec[3:15], rec[15:21] = d["com_des"][b], d["leg_des"][b], d["F_force_des"][b]
            rec[21:24], rec[24:27], rec[27:30] = d["rfoot_des"][b], d["lfoot_des"][b], d["base_p"][b]
            rec[30:42], rec[42:48], rec[48] = d["feet_p"][b], d["FT_total_des"][b], d["y_coef"][b]
            rec.tofile(f)
            np.array([d["mode"][b], d["right_support"][b]], np.int32).tofile(f)
    r = subprocess.run([os.path.join(ORACLE, "_build_asan", "asan_check"), str(tmp_path)],
                       capture_output=True, text=True, env=_env(), timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert "rt %d" % (T * B) in r.stdout
    del O


def test_oracle_cpu_tests_with_ubsan_library():
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True)
    tests = [os.path.join(ROOT, "tests", t) for t in
             ("test_oracle.py", "test_servo.py", "test_support_phase.py", "test_a1qp.py",
              "test_kin.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu"] + tests,
                       capture_output=True, text=True, env=_env(QLOCO_ORACLE_UBSAN="1"),
                       cwd=ROOT, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out, out[-4000:]


def test_host_shim_under_asan_ubsan():
    from quadrupedal_loco_amd import build as qb
    qb.build()
    outdir = os.path.join(ROOT, "tests", "cpp", "_build_asan")
    os.makedirs(outdir, exist_ok=True)
    exe = os.path.join(outdir, "host_asan")
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-gpu-sanitize",
           "-fno-omit-frame-pointer", "-g", "-O1"]
    cmd = ([qb.HIPCC, "-x", "c++", "-std=c++17", "-I" + qb.INCLUDE] + qb.HIP_HOST + san +
           [qb.HOST_SRC, os.path.join(ROOT, "tests", "cpp", "host_asan.cpp"), "-o", exe,
            "-L" + qb.LIBDIR, "-lqloco", "-Wl,-rpath," + qb.LIBDIR] + qb.HIP_LINK)
    subprocess.run(cmd, check=True, capture_output=True)
    env = _env(HIP_VISIBLE_DEVICES="")  # this host has no GPU; keep it that way on any host
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "host_asan ALL OK" in r.stdout, out[-4000:]
    assert "runtime error" not in out, out[-4000:]
