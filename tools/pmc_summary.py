"""Summarise rocprofv3 PMC databases written by tools/gpu_pmc.sh (per-wave averages)."""
import collections
import glob
import os
import sqlite3
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "srbd_admm"
for d in sorted(glob.glob(os.path.join(root, "pmc*_*"))):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        continue
    cur = sqlite3.connect(dbs[0]).cursor()
    rows = cur.execute("select kernel_name, counter_name, value from counters_collection").fetchall()
    agg = collections.defaultdict(list)
    for k, c, v in rows:
        if kern in str(k):
            agg[c].append(v)
    print(os.path.basename(d), {c: round(sum(v) / len(v)) for c, v in sorted(agg.items())})
