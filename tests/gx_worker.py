"""Worker for test_xg_adam_gpu.py: W processes share the GPU and train BASELINE's 3x128 weather
MLP through FusedMLPEngine's DDP step path with the fused peer all-reduce + Adam kernel
(csrc/xg_adam.hip) over IPC-mapped receive buffers.  gloo is the control plane (RCCL refuses two
ranks on one device), so the exchange is the only gradient path.  Rank 0 writes argv[1]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.models.mlp import MLPClassifier  # noqa: E402
from dct_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from dct_amd.trainer.engines import FusedMLPEngine, adam_hparams_from  # noqa: E402


def main():
    out_path, steps, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    # "step": the DDP step path (grad kernel + peer all-reduce/Adam kernel); "inkernel": the
    # persistent 3x128 launch with its own reduce-scatter / all-gather (csrc/mlp_block5.hip)
    path = sys.argv[4] if len(sys.argv) > 4 else "step"
    if path == "step":
        os.environ["DCT_XG_INKERNEL"] = "0"
    FusedMLPEngine.GRAPH_CHUNK = 16
    ctx = init_distributed("gpu", backend="gloo")
    X, Y = weather_tensors(3000, seed=1)
    rows = torch.randperm(3000, generator=torch.Generator().manual_seed(0))
    torch.manual_seed(0)
    model = MLPClassifier(5, hidden=(128, 128), dropout=0.0)
    eng = FusedMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
    eng.attach_data(X, Y, rows[:2400], rows[2400:])
    n = eng.upload_epoch_indices(0)
    local = eng.train_rows[eng.epoch_local_indices(len(eng.train_rows), 0, True)][: steps * B]
    loss = torch.zeros(steps, device=ctx.device)
    ctx.barrier()
    first = steps // 2 + 3  # two run_steps calls: graph replays + eager remainder in each
    eng.run_steps(n, first, loss, first_step=0)
    eng.run_steps(n, steps - first, loss, first_step=first)
    torch.cuda.synchronize()
    st = eng.xg_verify(fallback=False)
    res = {"mode": eng.step_mode, "gx": eng.gx is not None, "xg": eng.xg is not None, "graph_used": eng.graph_used,
           "ok": st, "step_counter": int(eng.step_counter.item()), "params": eng.p.cpu().tolist(),
           "m": eng.m.cpu().tolist(), "v": eng.v.cpu().tolist(), "losses": loss.cpu().tolist(),
           "rows": local.tolist()}
    allres = ctx.all_gather_object(res)
    if ctx.rank == 0:
        with open(out_path, "w") as f:
            json.dump(allres, f)
    ctx.barrier()
    del eng
    shutdown(ctx)


if __name__ == "__main__":
    main()
