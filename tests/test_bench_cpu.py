"""bench.py contract on the CPU plumbing config (BASELINE config 1): one JSON line with the
driver's keys, single process and a 2-rank gloo DDP run (replicas must stay in sync)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def test_bench_cpu_single_process_contract():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--steps", "40",
                        "--warmup", "5"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _last_json(r.stdout)
    assert KEYS <= set(out) and out["steps"] == 40 and out["warmup"] == 5 and out["value"] > 0
    assert out["config"]["global_batch"] == 4 and out["config"]["parallelism"] == "dp1-cpu-gloo"
    assert out["extra"]["losses_finite"] and out["extra"]["params_in_sync"]


@pytest.mark.slow
def test_bench_cpu_two_rank_gloo_ddp():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29661", os.path.join(ROOT, "bench.py"), "--device", "cpu",
           "--gpus", "2", "--steps", "30", "--warmup", "5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = _last_json(r.stdout)
    assert out["config"]["global_batch"] == 8 and out["config"]["parallelism"] == "dp2-cpu-gloo"
    assert out["extra"]["params_in_sync"] is True
