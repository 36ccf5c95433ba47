"""Per-SIMD end-time spread of the literal N = 10 kernel at the headline batch
(the tail the one-wave-per-instance launch waits on).

    python tools/simd_spread.py build          (CPU: builds tools/_var/spread/libqloco.so)
    QLOCO_LIB=tools/_var/spread/libqloco.so python tools/simd_spread.py run [B] [GAIT] [shuffle]   (GPU)

The variant (tools/variant_lib.py --patch, never the product library) wraps
srbd_lit_kernel: lane 0 of every workgroup reads the 100 MHz real-time
counter before and after the solve and the wave's hardware ids (HW_ID: SIMD
[5:4], CU [11:8], SH [12], SE [15:13]; XCC_ID), and writes them over the
first five floats of its own u row (vector stores) -- the u output of this
variant is therefore not the solution.  The run aggregates per SIMD: the
first start, the last end, the summed busy time, the number of waves it ran,
and prints the spread of the SIMD end times against the kernel span."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

OLD = """  if (i >= a.batch) return;
  srbd_lit_one<1, WS>(a, S, i);
}"""
NEW = """  if (i >= a.batch) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  srbd_lit_one<1, WS>(a, S, i);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  if (threadIdx.x == 0 && a.u) {
    unsigned *o = reinterpret_cast<unsigned *>(a.u + i * (12 * a.N));
    o[0] = (unsigned)t0; o[1] = (unsigned)(t0 >> 32);
    o[2] = (unsigned)t1; o[3] = (unsigned)(t1 >> 32);
    o[4] = hw; o[5] = xcc;
  }
}"""


def build():
    import variant_lib
    variant_lib.main(["spread", "--patch", "qloco_srbd_lit.hip:" + OLD + "=>" + NEW])


def run(B, gait, shuffle=False):
    import torch

    from quadrupedal_loco_amd import _lib, srbd
    if os.environ.get("QLOCO_LIB"):
        _lib.LIB_PATH = os.environ["QLOCO_LIB"]
    N = 10
    dev = torch.device("cuda:0")
    x0, xr, ft, ct = srbd.generate(20261015, N, B, gait)
    if shuffle:  # bench.py's shuffled_order line: the same seeded permutation
        perm = np.random.default_rng(20261015 + 1).permutation(B)
        x0, xr, ft, ct = (a[perm] for a in (x0, xr, ft, ct))
    args = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0, xr, ft, ct)]
    s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1)
    out = s.alloc_outputs(B, dev, full=True)
    for _ in range(60):  # past the clock ramp
        s.solve(*args, out=out, max_legs=4 * N)
    torch.cuda.synchronize()
    reps = []
    for _ in range(5):
        s.solve(*args, out=out, max_legs=4 * N)
        torch.cuda.synchronize()
        reps.append(out.u.view(torch.int32).cpu().numpy().reshape(B, 12 * N)[:, :6].astype(np.uint32))
    it = out.iters.cpu().numpy()
    for r, w in enumerate(reps):
        t0 = w[:, 0].astype(np.uint64) | (w[:, 1].astype(np.uint64) << np.uint64(32))
        t1 = w[:, 2].astype(np.uint64) | (w[:, 3].astype(np.uint64) << np.uint64(32))
        hw, xcc = w[:, 4], w[:, 5] & 0xF
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        key = (((xcc.astype(np.int64) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
        base = t0.min()
        s0 = (t0 - base).astype(np.float64) * 0.01  # 100 MHz ticks -> us
        s1 = (t1 - base).astype(np.float64) * 0.01
        span = s1.max()
        keys, inv = np.unique(key, return_inverse=True)
        end = np.zeros(len(keys))
        busy = np.zeros(len(keys))
        nw = np.zeros(len(keys), int)
        itsum = np.zeros(len(keys))
        np.maximum.at(end, inv, s1)
        np.add.at(busy, inv, s1 - s0)
        np.add.at(nw, inv, 1)
        np.add.at(itsum, inv, it)
        pct = np.percentile(end, [0, 10, 50, 90, 100])
        print("rep %d: B=%d %s%s  kernel span %.1f us  SIMDs used %d (XCCs %d)  waves/SIMD min %d max %d" % (
            r, B, gait, " shuffled" if shuffle else "", span, len(keys), len(np.unique(xcc)), nw.min(), nw.max()))
        print("   SIMD end time us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f;  mean SIMD idle tail %.1f us "
              "(%.1f%% of the span)" % (*pct, span - end.mean(), 100 * (span - end.mean()) / span))
        print("   per-wave solve us: p50 %.1f p99 %.1f max %.1f;  per-SIMD iterations sum min %d p50 %d max %d" % (
            *np.percentile(s1 - s0, [50, 99, 100]), itsum.min(), np.median(itsum), itsum.max()))
        if r == 0:
            # dispatch placement: do the instances sharing a SIMD follow i mod (number of SIMDs)?
            nsimd = len(keys)
            same = np.mean([len(set((np.nonzero(inv == k)[0] % nsimd).tolist())) == 1 for k in range(nsimd)])
            print("   placement: %.3f of SIMDs hold instances with one value of i mod %d; "
                  "SIMD key of instances 0..7: %s" % (same, nsimd, key[:8].tolist()))
            late = np.argsort(-end)[:3]
            for k in late:
                sel = inv == k
                print("   late SIMD key %d: %d waves, iterations %s, end %.1f us" % (
                    keys[k], nw[k], sorted(it[sel].tolist()), end[k]))
        sys.stdout.flush()


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 4096, sys.argv[3] if len(sys.argv) > 3 else "trot",
            len(sys.argv) > 4 and sys.argv[4] == "shuffle")
