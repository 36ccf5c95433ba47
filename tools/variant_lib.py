"""Build an experimental copy of libqloco.so with extra -D flags into
tools/_var/<name>/ (never the product library).  perf_kernel.py loads it
when QLOCO_LIB points at it.
    python tools/variant_lib.py NAME -DFOO=1 ...
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from quadrupedal_loco_amd import build as qb  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(HERE, "_var", name)
os.makedirs(out, exist_ok=True)
objs = []
for src in qb.SOURCES:
    path = os.path.join(qb.CSRC, src)
    obj = os.path.join(out, src + ".o")
    if src.endswith(".hip"):
        cmd = ([qb.HIPCC, "--offload-arch=" + qb.ARCH, "-x", "hip"] + qb.COMMON +
               qb.EXTRA.get(src, []) + flags + ["-c", path, "-o", obj])
    else:
        cmd = [qb.HIPCC, "-x", "c++"] + qb.COMMON + ["-ffp-contract=off", "-c", path, "-o", obj]
    subprocess.run(cmd, check=True)
    objs.append(obj)
lib = os.path.join(out, "libqloco.so")
subprocess.run([qb.HIPCC, "--offload-arch=" + qb.ARCH, "-shared", "-fPIC", "-o", lib] + objs, check=True)
for o in objs:
    os.remove(o)
print(lib)
