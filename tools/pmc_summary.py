"""Summarise rocprofv3 PMC databases: per dispatch, each counter summed over
its dimensions (SE / XCD instances), then averaged over the dispatches of the
matching kernel.  Usage: python tools/pmc_summary.py DIR [KERNEL_SUBSTRING]
(DIR: a rocprofv3 -d directory, or a parent holding pmc*/ subdirectories)."""
import collections
import glob
import os
import sqlite3
import sys


def summarise(d, kern):
    """{kernel name: {counter: mean over that kernel's dispatches}} for the
    kernels whose name contains `kern` (one entry per distinct kernel, so the
    classes of a multi-class SRBD batch are not averaged together)."""
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        return None
    cur = sqlite3.connect(dbs[0]).cursor()
    rows = cur.execute("select dispatch_id, kernel_name, counter_name, value, duration "
                       "from counters_collection").fetchall()
    per = collections.defaultdict(float)
    dur = collections.defaultdict(dict)
    for disp, k, c, v, du in rows:
        if kern in str(k):
            per[(str(k), disp, c)] += v
            dur[str(k)][disp] = du
    res = {}
    for name in sorted(dur):
        agg = collections.defaultdict(list)
        for (k, disp, c), v in per.items():
            if k == name:
                agg[c].append(v)
        out = {c: sum(v) / len(v) for c, v in sorted(agg.items())}
        out["duration_ns"] = sum(dur[name].values()) / len(dur[name])
        out["dispatches"] = len(dur[name])
        res[name] = out
    return res


if __name__ == "__main__":
    root = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "srbd_admm"
    dirs = [root] if glob.glob(os.path.join(root, "*.db")) or glob.glob(
        os.path.join(root, "*", "*.db")) and not glob.glob(os.path.join(root, "pmc*")) else \
        sorted(glob.glob(os.path.join(root, "pmc*")))
    for d in dirs:
        s = summarise(d, kern)
        for name, v in (s or {}).items():
            print(os.path.basename(d), name[:60], {k: round(x) for k, x in v.items()})
