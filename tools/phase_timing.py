"""Per-phase cycle counts of the SRBD kernel (development tool).

Builds a separate copy of libqloco.so with -DQLOCO_PHASE_TIMING into
tools/_phase/ (never the product library), runs one launch and prints the
mean / max cycles (s_memtime-style shader clock) at each phase boundary:
1 inputs+stance, 2 model+gradient, 3 P row, 4 Ruiz, 5 K finalize,
6 inverse, 7 ADMM loop, 8 outputs.
    python tools/phase_timing.py [variant] [B]
PHASE_NAME / PHASE_FLAGS (env) build and select a named copy with extra -D
flags (e.g. PHASE_NAME=row PHASE_FLAGS=-DQLOCO_SRBD_SPLIT=0).
"""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, "_phase", os.environ.get("PHASE_NAME", "prod"))
FLAGS = os.environ.get("PHASE_FLAGS", "").split()


def build():
    from quadrupedal_loco_amd import build as qb
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for src in qb.SOURCES:
        path = os.path.join(qb.CSRC, src)
        obj = os.path.join(OUT, src + ".o")
        if src.endswith(".hip"):
            cmd = ([qb.HIPCC, "--offload-arch=" + qb.ARCH, "-x", "hip"] + qb.COMMON +
                   qb.EXTRA.get(src, []) + ["-DQLOCO_PHASE_TIMING"] + FLAGS + ["-c", path, "-o", obj])
        else:
            cmd = [qb.HIPCC, "-x", "c++"] + qb.COMMON + ["-ffp-contract=off", "-c", path, "-o", obj]
        subprocess.run(cmd, check=True)
        objs.append(obj)
    lib = os.path.join(OUT, "libqloco.so")
    subprocess.run([qb.HIPCC, "--offload-arch=" + qb.ARCH, "-shared", "-fPIC", "-o", lib] + objs,
                   check=True)
    return lib


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        print(build())
        sys.exit(0)
    import numpy as np
    import torch
    from quadrupedal_loco_amd import _lib, srbd
    _lib.LIB_PATH = os.path.join(OUT, "libqloco.so")
    sys.path.insert(0, HERE)
    from perf_kernel import VARIANTS
    name = sys.argv[1] if len(sys.argv) > 1 else "default"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    N = 10
    x0, xr, ft, ct = srbd.generate(20261015, N, B, "trot")
    dev = torch.device("cuda:0")
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    s = srbd.BatchedConvexMpc(horizon=N, **VARIANTS[name])
    out = s.alloc_outputs(B, dev)
    for _ in range(3):
        s.solve(*args, out=out, max_legs=srbd.max_stance_legs(ct, N))
    torch.cuda.synchronize()
    buf = np.zeros(min(B, 1 << 16) * 16, np.uint32)
    dl = C.CDLL(_lib.LIB_PATH)
    rc = dl.qloco_phase_read(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.size))
    if rc != 0:
        raise SystemExit("qloco_phase_read failed %d" % rc)
    ph = buf.reshape(-1, 16)[:, :9].astype(np.float64)
    d = np.diff(ph[:, 1:9], axis=1, prepend=0.0)
    labels = ["inputs+stance", "model+gradient", "P row", "Ruiz", "K finalize", "inverse",
              "ADMM loop", "outputs"]
    it = out.iters.cpu().numpy()
    print("%s variant %s B=%d  mean iters %.1f max %d" % (os.environ.get("PHASE_NAME", "prod"), name, B, it.mean(), it.max()))
    for k, lab in enumerate(labels):
        print("  %-16s mean %9.0f  max %9.0f cycles" % (lab, d[:, k].mean(), d[:, k].max()))
    print("  %-16s mean %9.0f  max %9.0f cycles" % ("TOTAL", ph[:, 8].mean(), ph[:, 8].max()))
    sub = buf.reshape(-1, 16)[:, 9:].astype(np.float64)
    for k, lab in enumerate(["ruiz head", "ruiz absmax", "ruiz reduce", "sub12", "sub13", "sub14", "sub15"]):
        if sub[:, k].any():
            print("  %-16s mean %9.0f  max %9.0f cycles (sum over passes)" % (lab, sub[:, k].mean(), sub[:, k].max()))
