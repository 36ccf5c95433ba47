#!/bin/bash
# One parameterised GPU launcher (run through gpurun from the repo root):
#   tools/gpu.sh TAG STEP [STEP ...]
# Every step writes under gpurun_out/TAG/, runs under its own time limit and
# stops the call on the first failure (no GPU step after a failed one).
# Steps:
#   tests        pytest -m gpu (parity suite)            -> pytest_gpu.log
#   tk=EXPR      pytest -m gpu -k EXPR                   -> pytest_k.log
#   smoke        __graft_entry__.smoke()                 -> smoke.log
#   bench        python bench.py (default line)          -> bench.json
#   ktrace       rocprofv3 --kernel-trace --stats of the bench -> kernel_stats.csv
#   ktraceh      headline-only kernel trace (--no-second-line), last 50 launches -> kernel_stats_headline.csv
#   sq[=VAR]     two SQ counter passes of perf_kernel.py VAR (default; env N, GAIT, LITERAL, TB = batch)
#                                                         -> pmc_sq_n*_b*_lit*.txt
#   sqqp[=ARGS]  two SQ counter passes of the grouped force-QP launch (tools/bench_qp.py) -> pmc_sq_qp.txt
#   traffic[=VAR] FETCH_SIZE / WRITE_SIZE passes (env as sq) -> traffic_*.json
#   configs      bench lines of configs 3-5 (per-GPU shares) -> configs.jsonl
#   lit          literal-QP lines at N = 10 / 16 / 20     -> literal.jsonl
#   breakdown    perf_kernel.py ablations (setup / iterations / checks), reduced + literal
#   scan         batch-size scan of the default kernel    -> scan.txt
#   qp / rt      force-QP and rt-tick bench lines         -> bench_qp.json / bench_rt.json
#   probe=NAME   tools/micro/NAME (prebuilt)              -> probe_NAME.txt
#   ab=LIBS      perf_kernel default + bench per library (comma list of
#                tools/_var/NAME or "cur")                -> ab.txt
#   py=SCRIPT[:ARGS] python SCRIPT ARGS (ARGS ':'-separated) -> py_<script>.txt
# Environment passes through (N, GAIT, LITERAL, QLOCO_LIB ... for perf_kernel).
set -o pipefail
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1

fail() { tail -30 "$1"; exit 1; }

for step in "$@"; do
  name=${step%%=*}
  arg=""
  [[ $step == *=* ]] && arg=${step#*=}
  echo "== $step $(date +%T)"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$out/pytest_gpu.log" 2>&1 || fail "$out/pytest_gpu.log"
      tail -n 1 "$out/pytest_gpu.log" ;;
    tk)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${arg//:/ }" \
        > "$out/pytest_k.log" 2>&1 || fail "$out/pytest_k.log"
      tail -n 1 "$out/pytest_k.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
        || fail "$out/smoke.log"
      cat "$out/smoke.log" ;;
    bench)
      timeout -k 10 300 python bench.py ${arg//:/ } > "$out/bench.json" 2> "$out/bench.err" || fail "$out/bench.err"
      cat "$out/bench.json" ;;
    ktrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/ktrace" -o run -- python bench.py --steps 50 --warmup 5 \
        --no-cpu-baseline ${arg//:/ } > "$out/ktrace.log" 2>&1 || fail "$out/ktrace.log"
      python tools/db_kernel_stats.py "$out/ktrace" > "$out/kernel_stats.csv" && rm -rf "$out/ktrace"
      head -5 "$out/kernel_stats.csv" ;;
    ktraceh)
      # headline only (no side lines), stats over the K timed launches
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/ktraceh" -o run -- python bench.py --steps 50 --warmup 5 \
        --no-second-line --no-cpu-baseline ${arg//:/ } > "$out/ktraceh.log" 2>&1 || fail "$out/ktraceh.log"
      python tools/db_kernel_stats.py "$out/ktraceh" --last 50 > "$out/kernel_stats_headline.csv" && rm -rf "$out/ktraceh"
      head -5 "$out/kernel_stats_headline.csv"; tail -1 "$out/ktraceh.log" ;;
    sq)
      v=${arg:-default}
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d "$out/pmc1" -o run -- python tools/perf_kernel.py "$v" ${TB:-4096} 3 \
        > "$out/pmc1.log" 2>&1 || fail "$out/pmc1.log"
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM \
        SQ_INSTS_SALU GRBM_GUI_ACTIVE -d "$out/pmc2" -o run -- python tools/perf_kernel.py "$v" ${TB:-4096} 3 \
        > "$out/pmc2.log" 2>&1 || fail "$out/pmc2.log"
      sqf="$out/pmc_sq_n${N:-10}_${GAIT:-trot}_b${TB:-4096}_lit${LITERAL:-0}.txt"
      python tools/pmc_summary.py "$out/pmc1" srbd > "$sqf" && python tools/pmc_summary.py "$out/pmc2" srbd >> "$sqf"
      rm -rf "$out/pmc1" "$out/pmc2"
      cat "$sqf" ;;
    sqqp)
      # SQ counters of the grouped force-QP launch (tools/bench_qp.py, 65,536 robots)
      for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
               "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
        n=$((n + 1))
        timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $p -d "$out/pmcq$n" -o run -- python tools/bench_qp.py \
          --steps 3 --warmup 2 --no-cpu-baseline ${arg//:/ } > "$out/pmcq$n.log" 2>&1 || fail "$out/pmcq$n.log"
        python tools/pmc_summary.py "$out/pmcq$n" force_qp >> "$out/pmc_sq_qp.txt"
        rm -rf "$out/pmcq$n"
      done
      cat "$out/pmc_sq_qp.txt" ;;
    traffic)
      v=${arg:-default}
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/fetch" -o run -- python tools/perf_kernel.py "$v" ${TB:-4096} 3 \
        > "$out/fetch.log" 2>&1 || fail "$out/fetch.log"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$out/write" -o run -- python tools/perf_kernel.py "$v" ${TB:-4096} 3 \
        > "$out/write.log" 2>&1 || fail "$out/write.log"
      python tools/prof_summary.py traffic "$out/fetch" "$out/write" srbd "$out/traffic_${v}_n${N:-10}_${GAIT:-trot}_b${TB:-4096}_lit${LITERAL:-0}.json"
      rm -rf "$out/fetch" "$out/write" ;;
    configs)
      for spec in "16 trot 65536" "20 pace 65536" "10 mixed 131072"; do
        set -- $spec
        timeout -k 10 240 python bench.py --horizon $1 --gait $2 --batch $3 --steps 20 --warmup 3 --no-cpu-baseline \
          >> "$out/configs.jsonl" 2>> "$out/configs.err" || fail "$out/configs.err"
      done
      cat "$out/configs.jsonl" ;;
    lit)
      for spec in "10 trot 4096" "10 mixed 131072" "16 trot 8192" "20 pace 8192"; do
        set -- $spec
        N=$1 GAIT=$2 LITERAL=1 timeout -k 10 120 python tools/perf_kernel.py default $3 10 >> "$out/literal.txt" 2>&1 \
          || fail "$out/literal.txt"
      done
      grep -v amdgpu.ids "$out/literal.txt" ;;
    breakdown)
      for lit in 0 1; do
        for v in default iter0 iter0s0 iter150 chk5; do
          LITERAL=$lit timeout -k 10 120 python tools/perf_kernel.py $v 4096 10 >> "$out/breakdown.txt" 2>&1 \
            || fail "$out/breakdown.txt"
        done
      done
      grep -v amdgpu.ids "$out/breakdown.txt" ;;
    scan)
      for b in 1 1024 2048 4096 8192 16384 65536; do
        timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> "$out/scan.txt" 2>&1 || fail "$out/scan.txt"
      done
      grep -v amdgpu.ids "$out/scan.txt" ;;
    qp)
      timeout -k 10 200 python tools/bench_qp.py ${arg//:/ } > "$out/bench_qp.json" 2> "$out/bench_qp.err" || fail "$out/bench_qp.err"
      cat "$out/bench_qp.json" ;;
    rt)
      timeout -k 10 200 python tools/bench_rt.py > "$out/bench_rt.json" 2> "$out/bench_rt.err" || fail "$out/bench_rt.err"
      cat "$out/bench_rt.json" ;;
    probe)
      timeout -k 10 120 "tools/micro/$arg" > "$out/probe_$arg.txt" 2>&1 || fail "$out/probe_$arg.txt"
      cat "$out/probe_$arg.txt" ;;
    ab)
      IFS=, read -ra libs <<< "$arg"
      for lib in "${libs[@]}"; do
        if [ "$lib" = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=$lib/libqloco.so; fi
        timeout -k 10 120 python tools/perf_kernel.py default 4096 20 2>&1 | grep -v amdgpu.ids | sed "s|^|$lib |" >> "$out/ab.txt" \
          || fail "$out/ab.txt"
      done
      unset QLOCO_LIB
      cat "$out/ab.txt" ;;
    py)
      script=${arg%%:*}
      rest=""
      [[ $arg == *:* ]] && rest=${arg#*:}
      timeout -k 10 600 python -u "$script" ${rest//:/ } > "$out/py_$(basename "$script" .py).txt" 2>&1 \
        || fail "$out/py_$(basename "$script" .py).txt"
      tail -40 "$out/py_$(basename "$script" .py).txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
