"""rocprofv3 kernel-trace database -> the --stats kernel_stats.csv layout
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).
    python tools/db_kernel_stats.py DB_DIR > profiles/NAME_kernel_stats.csv
"""
import collections
import glob
import sqlite3
import sys

import numpy as np

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
rows = sqlite3.connect(db).cursor().execute("select name, start, end from kernels").fetchall()
d = collections.defaultdict(list)
for name, s, e in rows:
    d[name].append(e - s)
tot = sum(sum(v) for v in d.values())
print("Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs,StdDev")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    a = np.array(v, dtype=np.float64)
    print('"%s",%d,%d,%.1f,%.3f,%d,%d,%.1f' % (k, len(v), a.sum(), a.mean(), 100 * a.sum() / tot,
                                              a.min(), a.max(), a.std()))
