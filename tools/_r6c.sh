#!/bin/bash
set -o pipefail
out=gpurun_out/r6c; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
for id in 5 12 0; do
  QSET=isaac timeout -k 10 120 python tools/lit_dump_t.py run 16 trot $id 0.1 1e-2 1e-3 1e-4 >> $out/dump.txt 2>&1 || { tail $out/dump.txt; exit 1; }
done
timeout -k 10 120 python tools/lit_dump_t.py run 16 trot 5 0.1 1e-3 >> $out/dump.txt 2>&1 || { tail $out/dump.txt; exit 1; }
QSET=isaac timeout -k 10 120 python tools/lit_dump_t.py run 10 trot 5 0.1 1e-3 >> $out/dump.txt 2>&1 || { tail $out/dump.txt; exit 1; }
grep -v amdgpu.ids $out/dump.txt
