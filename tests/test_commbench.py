"""All-reduce microbenchmark (parallel/commbench.py): size sweep, busBW arithmetic, knee, and a
2-rank gloo run through the same CLI the 8-GPU RCCL sweep uses (tools/bench_allreduce.py)."""
import json
import os
import subprocess
import sys

import dct_amd  # noqa: F401
from dct_amd.parallel.commbench import bucket_knee, bus_factor, format_table, sizes_pow2

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sizes_and_bus_factor():
    assert sizes_pow2(8, 64) == [8, 16, 32, 64]
    assert sizes_pow2(1, 4) == [4]
    assert bus_factor(1) == 0.0
    assert bus_factor(2) == 1.0
    assert abs(bus_factor(8) - 1.75) < 1e-12


def test_bucket_knee_and_table():
    recs = [{"path": "native", "bytes": b, "world": 8, "us": 1.0, "algbw_GBps": bw / 1.75, "busbw_GBps": bw,
             "correct": True, "dtype": "fp32"} for b, bw in [(1 << 10, 1.0), (1 << 20, 60.0), (1 << 23, 290.0),
                                                              (1 << 26, 330.0)]]
    assert bucket_knee(recs, "native") == 1 << 23  # first size >= 80 % of 330 GB/s
    assert bucket_knee(recs, "torch") is None
    assert "native" in format_table(recs)


def test_two_rank_gloo_sweep_is_correct():
    e = dict(os.environ)
    e.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29641", os.path.join(ROOT, "tools", "bench_allreduce.py"),
           "--accelerator", "cpu", "--max-bytes", "65536", "--iters", "3", "--warmup", "1", "--json"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [x["bytes"] for x in recs] == sizes_pow2(8, 65536)
    assert all(x["correct"] and x["world"] == 2 and x["path"] == "torch" for x in recs)
    assert all(x["busbw_GBps"] == x["algbw_GBps"] for x in recs)  # factor 1 at W = 2


import pytest  # noqa: E402


@pytest.mark.gpu
def test_native_and_graph_paths_on_device():
    """W = 1 on one MI355X: the C++ RCCL communicator, eager and captured in a HIP graph."""
    import torch

    from dct_amd.parallel.commbench import run
    from dct_amd.parallel.dist import DistContext

    ctx = DistContext(device=torch.device("cuda", 0))
    recs = run(ctx, sizes_pow2(8, 1 << 20), "fp32", ("torch", "native", "graph"), iters=5, warmup=1)
    assert len(recs) == 3 * len(sizes_pow2(8, 1 << 20))
    assert all(r["correct"] and r["us"] > 0 for r in recs)
    recs = run(ctx, [4096], "bf16", ("native",), iters=2, warmup=1)
    assert recs[0]["correct"] and recs[0]["bytes"] == 4096


@pytest.mark.gpu
def test_one_rank_collectives_are_the_identity(monkeypatch):
    """A one-rank communicator skips in-place all-reduce / broadcast (RCCL's one-rank path is a
    pre-multiply kernel plus blits for the identity); DCT_RCCL_ONE_RANK=1 calls RCCL - both leave
    the buffer bit-identical."""
    import torch

    from dct_amd.ops._native import native

    nat = native()
    x = torch.randn(10_001, device="cuda")
    for force in ("0", "1"):
        monkeypatch.setenv("DCT_RCCL_ONE_RANK", force)
        comm = nat.Comm(nat.comm_unique_id(), 1, 0, 0)
        y = x.clone()
        st = torch.cuda.current_stream().cuda_stream
        comm.allreduce(y.data_ptr(), y.numel(), nat.DT_F32, nat.OP_AVG, st)
        comm.allreduce(y.data_ptr(), y.numel(), nat.DT_F32, nat.OP_SUM, st)
        comm.broadcast(y.data_ptr(), y.numel(), nat.DT_F32, 0, st)
        torch.cuda.synchronize()
        assert torch.equal(x, y), force
        del comm
    monkeypatch.delenv("DCT_RCCL_ONE_RANK")
    nat.reload_knobs()
