#!/bin/bash
# Round-3 run C: literal rho diagnostic, phase clocks of the headline kernel,
# new GPU tests (wide EiQuadProg, two streams, graph capture, literal mode).
set -o pipefail
tag=${1:-r3c}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/literal_rho_diag.py > $out/rho_diag.txt 2>&1 || { tail -20 $out/rho_diag.txt; exit 1; }
cat $out/rho_diag.txt
for b in 1 4096; do
  timeout -k 10 120 python tools/phase_timing.py default $b >> $out/phase.txt 2>&1 || { tail -20 $out/phase.txt; exit 1; }
done
cat $out/phase.txt
timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py tests/test_srbd_gpu.py tests/test_host_gpu.py -v --timeout 300 --timeout-method thread -k "wide or stream or graph or literal or cpp" > $out/pytest.log 2>&1; grep -E "PASS|FAIL|passed|failed" $out/pytest.log | tail -40
