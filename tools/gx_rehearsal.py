"""Per-step time of the 3x128 DDP step path with the fused peer all-reduce + Adam kernel
(csrc/xg_adam.hip) for W ranks SHARING one GPU (IPC-mapped buffers, gloo control plane; no xGMI
links involved, so this prices the kernels and the exchange protocol, not the fabric).

  python -m torch.distributed.run --nnodes=1 --nproc-per-node=W --master-addr=127.0.0.1 \\
      --master-port=29600 tools/gx_rehearsal.py [steps] [warmup]

Rank 0 prints one line: W, us/step over the timed window (barrier + device sync on both sides,
max over ranks) and whether the replicas are bit-identical afterwards."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.models.mlp import MLPClassifier  # noqa: E402
from dct_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from dct_amd.trainer.engines import FusedMLPEngine, adam_hparams_from  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ctx = init_distributed("gpu", backend="gloo")
    B = 4
    rows = (steps + warmup + 8) * B * ctx.world_size * 5 // 4 + 1024
    X, Y = weather_tensors(rows, seed=0)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    torch.manual_seed(0)
    model = MLPClassifier(5, hidden=(128, 128), dropout=0.0)
    eng = FusedMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
    eng.attach_data(X, Y, perm[: int(0.8 * rows)], perm[int(0.8 * rows):])
    n = eng.upload_epoch_indices(0)
    loss = torch.zeros(steps + warmup, device=ctx.device)
    eng.run_steps(n, warmup, loss, first_step=0)
    eng._get_graph(n, min(eng.graph_chunk, steps), loss)
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    eng.run_steps(n, steps, loss, first_step=warmup)
    torch.cuda.synchronize()
    ctx.barrier()
    dt = ctx.all_reduce_max_int(int((time.perf_counter() - t0) * 1e9)) * 1e-9
    ok = eng.xg_verify(fallback=False)
    ps = ctx.all_gather_object(eng.p.cpu())
    same = all(torch.equal(p, ps[0]) for p in ps)
    if ctx.rank == 0:
        print(f"W={ctx.world_size} mode={eng.step_mode} {dt / steps * 1e6:.2f} us/step "
              f"status_ok={ok} replicas_identical={same} loss_last={float(loss[-1]):.4f}", flush=True)
    ctx.barrier()
    del eng
    shutdown(ctx)


if __name__ == "__main__":
    main()
