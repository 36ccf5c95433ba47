"""Build libqloco.so (HIP, gfx950) in-tree with hipcc.

No cmake / JIT: one hipcc line per translation unit, objects cached by
mtime under quadrupedal_loco_amd/lib/obj/, linked into
quadrupedal_loco_amd/lib/libqloco.so (git-ignored, travels to the GPU box).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libqloco.so")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = [
    "qloco_capi.hip",
    "qloco_srbd.hip",
    "qloco_srbd_lit.hip",
    "qloco_srbd_build.hip",
    "qloco_kin.hip",
    "qloco_gi.hip",
    "qloco_gi_wide.hip",
    "qloco_force.hip",
    "qloco_body.hip",
    "qloco_rt.hip",
    "qloco_servo.hip",
    "qloco_a1qp.hip",
    "qloco_mgpu.hip",
    "qloco_gen.cpp",
]
# per-file extra flags: the fp64 active-set kernel keeps the restatement's
# exact operation sequence (no FMA contraction)
# The SRBD kernel keeps a 64-wide register row per lane: SLP vectorisation
# pairs unrelated columns across the unrolled row loops and inflates live
# ranges into scratch spills, so it is off there (the packed-fp32 matvec and
# Gauss-Jordan updates are written with explicit float2 ops).  Its pivot
# loops are unrolled in full (static register per pivot column); the two-wave
# inverse's body exceeds the default pragma-unroll budget, so it is raised.
EXTRA = {"qloco_a1qp.hip": ["-ffp-contract=off"], "qloco_gi.hip": ["-ffp-contract=off"], "qloco_gi_wide.hip": ["-ffp-contract=off"], "qloco_force.hip": ["-ffp-contract=off"],
         "qloco_body.hip": ["-ffp-contract=off"], "qloco_rt.hip": ["-ffp-contract=off"], "qloco_servo.hip": ["-ffp-contract=off"], "qloco_kin.hip": ["-ffp-contract=off"], "qloco_srbd.hip": ["-fno-slp-vectorize", "-mllvm", "-pragma-unroll-threshold=200000"],
         "qloco_srbd_lit.hip": ["-fno-slp-vectorize", "-mllvm", "-pragma-unroll-threshold=200000"]}

COMMON = ["-O3", "-std=c++17", "-fPIC", "-I" + INCLUDE, "-I" + CSRC]


def _needs(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, jobs=8):
    os.makedirs(OBJDIR, exist_ok=True)
    headers = [os.path.join(INCLUDE, "qloco.h")] + [
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h", ".inc"))]
    cmds, objs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJDIR, src + ".o")
        objs.append(obj)
        if not _needs(obj, [path] + headers):
            continue
        if src.endswith(".hip"):
            cmd = ([HIPCC, "--offload-arch=" + ARCH, "-x", "hip"] + COMMON + EXTRA.get(src, []) +
                   ["-c", path, "-o", obj])
        else:  # host-only C++ (generator): exact IEEE, no contraction
            cmd = [HIPCC, "-x", "c++"] + COMMON + ["-ffp-contract=off", "-c", path, "-o", obj]
        cmds.append(cmd)
    procs = []
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        while len([p for _, p in procs if p.poll() is None]) >= jobs:
            procs[0][1].wait()
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError("hipcc failed: " + " ".join(cmd))
    if cmds or not os.path.exists(LIB) or _needs(LIB, objs):
        link = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-ldl"]
        if verbose:
            print(" ".join(link))
        subprocess.run(link, check=True)
    build_host(verbose)
    return LIB


HOST_SRC = os.path.join(HERE, "host", "qloco_host.cpp")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
# host-only C++ against the HIP runtime (no device code in these TUs)
HIP_HOST = ["-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include")]
HIP_LINK = ["-L" + os.path.join(ROCM, "lib"), "-lamdhip64"]
HOST_LIB = os.path.join(LIBDIR, "libqloco_host.so")


def build_host(verbose=False):
    """C++ shim with the reference's class signatures (include/qloco.hpp) ->
    libqloco_host.so, linked against libqloco.so (rpath $ORIGIN)."""
    deps = [HOST_SRC, os.path.join(INCLUDE, "qloco.hpp"), os.path.join(INCLUDE, "qloco.h"), LIB]
    if not _needs(HOST_LIB, deps):
        return HOST_LIB
    cmd = [HIPCC, "-x", "c++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I" + INCLUDE] + HIP_HOST + [
           HOST_SRC, "-o", HOST_LIB, "-L" + LIBDIR, "-lqloco", "-Wl,-rpath,$ORIGIN"] + HIP_LINK
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return HOST_LIB


def build_host_test(oracle_lib, verbose=False):
    """tests/cpp/test_host (test infrastructure: links the oracle as checker)."""
    src = os.path.join(ROOT, "tests", "cpp", "test_host.cpp")
    outdir = os.path.join(ROOT, "tests", "cpp", "_build")
    os.makedirs(outdir, exist_ok=True)
    exe = os.path.join(outdir, "test_host")
    if not _needs(exe, [src, HOST_LIB, LIB, oracle_lib]):
        return exe
    cmd = [HIPCC, "-x", "c++", "-O2", "-std=c++17", "-I" + INCLUDE] + HIP_HOST + [
           "-I" + os.path.join(ROOT, "oracle"), src, "-o", exe, "-L" + LIBDIR, "-lqloco_host",
           "-lqloco", "-L" + os.path.dirname(oracle_lib), "-lqloco_oracle",
           "-Wl,-rpath,$ORIGIN/../../../quadrupedal_loco_amd/lib",
           "-Wl,-rpath,$ORIGIN/../../../oracle/_build"] + HIP_LINK
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return exe


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
