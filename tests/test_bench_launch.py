"""bench.py's multi-rank launch path on CPU (gloo).

`python bench.py --gpus N` without a launcher must start N ranks itself (the
driver's scaling runs read n_gpus from the JSON line), and a rank whose
WORLD_SIZE disagrees with --gpus must refuse to run.  `--dist-selftest`
replaces the GPU solve by the step's one collective (the u0 all-gather in
rank order), so the whole launch path runs here without a GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          env=env, timeout=180)


@pytest.mark.parametrize("n", [1, 2])
def test_bench_gpus_n_launches_n_ranks(n):
    p = _run(["--gpus", str(n), "--dist-selftest"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == n
    assert res["requested"] == n
    assert res["allgather_ok"] is True


def test_bench_rejects_world_size_mismatch():
    p = _run(["--gpus", "4", "--dist-selftest"],
             {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in p.stderr


def test_usable_cores_and_cpu_model():
    sys.path.insert(0, ROOT)
    import bench
    n = bench.usable_cores()
    assert 1 <= n <= (os.cpu_count() or 1)
    assert isinstance(bench.cpu_model(), str) and bench.cpu_model()
