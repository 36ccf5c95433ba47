"""rocprofv3 kernel-trace database -> the --stats kernel_stats.csv layout
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).
    python tools/db_kernel_stats.py DB_DIR [--last K] > profiles/NAME_kernel_stats.csv
--last K keeps each kernel's last K dispatches (by start time): under
`bench.py --no-second-line --steps K` those are exactly the K timed steps of
the headline (the pre-warm and warm-up launches come first).
"""
import collections
import glob
import sqlite3
import sys

import numpy as np

args = sys.argv[1:]
last = None
if "--last" in args:
    i = args.index("--last")
    last = int(args[i + 1])
    del args[i:i + 2]
db = glob.glob(args[0] + "/**/*.db", recursive=True)[0]
rows = sqlite3.connect(db).cursor().execute("select name, start, end from kernels order by start").fetchall()
d = collections.defaultdict(list)
for name, s, e in rows:
    d[name].append(e - s)
if last:
    d = {k: v[-last:] for k, v in d.items()}
tot = sum(sum(v) for v in d.values())
print("Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs,StdDev")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    a = np.array(v, dtype=np.float64)
    print('"%s",%d,%d,%.1f,%.3f,%d,%d,%.1f' % (k, len(v), a.sum(), a.mean(), 100 * a.sum() / tot,
                                              a.min(), a.max(), a.std()))
