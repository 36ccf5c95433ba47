"""Steady-state per-kernel dispatch times from a rocprofv3 kernel-trace
database: mean / min / max of the last N dispatches of each kernel (the
rocprofv3 --stats averages mix warm-up dispatches in).
    python tools/steady_kernels.py DB_DIR [N]
"""
import collections
import glob
import sqlite3
import sys

import numpy as np

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sqlite3.connect(db).cursor().execute(
    "select name, start, end from kernels order by start").fetchall()
d = collections.defaultdict(list)
for name, s, e in rows:
    d[name.split("(")[0]].append((e - s) / 1e3)
for k, v in d.items():
    if len(v) <= n:
        continue
    t = np.array(v[-n - 1:-1])
    print("%-40s dispatches %4d  last %d: mean %7.1f us  min %7.1f  max %7.1f"
          % (k, len(v), n, t.mean(), t.min(), t.max()))
