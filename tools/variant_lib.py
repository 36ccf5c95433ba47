"""Build an experimental copy of libqloco.so into tools/_var/<name>/ (never
the product library).  perf_kernel.py / bench.py load it when QLOCO_LIB
points at it.

    python tools/variant_lib.py NAME [--rev REV] [--patch FILE:OLD=>NEW ...] [-DFOO=1 ...]

--rev REV   build the kernel sources of git revision REV instead of the work
            tree.  The product sources carry no experiment hooks; the round-3
            instrumentation (QLOCO_PHASE_TIMING, QLOCO_TRACE_SIMD,
            QLOCO_DEBUG_INST, QLOCO_ABLATE_*, QLOCO_GI_PHASE_TIMING,
            QLOCO_MATVEC4, the *_WPE occupancy macros) lives at revision
            5561824 and is reached as
                python tools/variant_lib.py phase --rev 5561824 -DQLOCO_PHASE_TIMING
--patch     a literal text substitution applied to csrc/FILE of the copy
            (OLD must occur exactly once): one-off experiments without
            touching the product source, e.g.
                --patch 'qloco_srbd.hip:constexpr int kShortWpe = 4;=>constexpr int kShortWpe = 3;'
-D...       extra compiler flags for the HIP translation units.
"""
import os
import shutil
import subprocess
import sys
import tarfile
import io

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from quadrupedal_loco_amd import build as qb  # noqa: E402


def main(argv):
    name = argv[0]
    rev, patches, flags = None, [], []
    i = 1
    while i < len(argv):
        if argv[i] == "--rev":
            rev = argv[i + 1]
            i += 2
        elif argv[i] == "--patch":
            patches.append(argv[i + 1])
            i += 2
        else:
            flags.append(argv[i])
            i += 1
    out = os.path.join(HERE, "_var", name)
    src_root = os.path.join(out, "src")
    if os.path.isdir(src_root):
        shutil.rmtree(src_root)
    os.makedirs(src_root)
    if rev:
        blob = subprocess.run(["git", "-C", ROOT, "archive", rev, "quadrupedal_loco_amd/csrc", "include"],
                              check=True, capture_output=True).stdout
        tarfile.open(fileobj=io.BytesIO(blob)).extractall(src_root)
    else:
        shutil.copytree(qb.CSRC, os.path.join(src_root, "quadrupedal_loco_amd", "csrc"))
        shutil.copytree(qb.INCLUDE, os.path.join(src_root, "include"))
    csrc = os.path.join(src_root, "quadrupedal_loco_amd", "csrc")
    inc = os.path.join(src_root, "include")
    for p in patches:
        fname, rule = p.split(":", 1)
        old, new = rule.split("=>", 1)
        path = os.path.join(csrc, fname)
        text = open(path).read()
        if text.count(old) != 1:
            raise SystemExit("patch %r: %d matches in %s" % (old, text.count(old), fname))
        open(path, "w").write(text.replace(old, new))
    common = [f for f in qb.COMMON if not f.startswith("-I")] + ["-I" + inc, "-I" + csrc]
    sources = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".cpp")))
    objs, procs = [], []
    for src in sources:
        path = os.path.join(csrc, src)
        obj = os.path.join(out, src + ".o")
        if src.endswith(".hip"):
            cmd = ([qb.HIPCC, "--offload-arch=" + qb.ARCH, "-x", "hip"] + common +
                   qb.EXTRA.get(src, []) + flags + ["-c", path, "-o", obj])
        else:
            cmd = [qb.HIPCC, "-x", "c++"] + common + ["-ffp-contract=off", "-c", path, "-o", obj]
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
        if len(procs) >= int(os.environ.get("MAX_JOBS", 6)):
            if procs.pop(0).wait() != 0:
                raise SystemExit("compile failed")
    for pr in procs:
        if pr.wait() != 0:
            raise SystemExit("compile failed")
    lib = os.path.join(out, "libqloco.so")
    subprocess.run([qb.HIPCC, "--offload-arch=" + qb.ARCH, "-shared", "-fPIC", "-o", lib] + objs, check=True)
    for o in objs:
        os.remove(o)
    print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
