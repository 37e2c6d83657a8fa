"""Worker for test_xgmi_gpu.py: W processes on the available GPU(s) train with the in-kernel
all-reduce over IPC-mapped receive buffers (gloo is the control plane: RCCL refuses two ranks
on one device).  Rank 0 writes the result JSON to argv[1]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.sampler import distributed_indices  # noqa: E402
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.ops.fused_mlp import FusedMLPKernel  # noqa: E402
from dct_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from dct_amd.parallel.xgmi import check, setup_peer_exchange  # noqa: E402


def main():
    out_path, steps, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    os.environ["DCT_ALLREDUCE"] = "xgmi"
    ctx = init_distributed("gpu", backend="gloo")
    dims = [5, 64, 2]
    kern = FusedMLPKernel(dims, bmax=4 if B <= 4 else 16)
    xg = setup_peer_exchange(kern, ctx, B)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(5, 64), torch.nn.ReLU(), torch.nn.Linear(64, 2))
    p = torch.cat([t.detach().reshape(-1) for t in net.state_dict().values()]).to(ctx.device)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    X, Y = weather_tensors(4000, seed=3)
    shard = distributed_indices(4000, ctx.world_size, ctx.rank, shuffle=True, seed=42, epoch=0)
    n_items = shard.numel()
    sc = torch.zeros(1, dtype=torch.int32, device=ctx.device)
    loss = torch.zeros(steps, device=ctx.device)
    ctx.barrier()
    kern.train(p, m, v, X.to(ctx.device), Y.to(ctx.device, torch.int32), shard.to(ctx.device, torch.int32),
               n_items=n_items, batch=B, steps=steps, t0=0, lr=0.01, loss_out=loss, step_counter=sc, xg=xg,
               xg_timeout_s=10.0)
    torch.cuda.synchronize()
    # device-side barrier: rank r arrives r x 30 ms late; nobody may leave before the last arrival
    import time

    from dct_amd.parallel.xgmi import device_barrier

    bar = []
    for _ in range(3):
        ctx.barrier()
        time.sleep(0.03 * ctx.rank)
        t_arrive = time.time()
        device_barrier(xg, torch.cuda.current_stream().cuda_stream, 10.0)
        torch.cuda.synchronize()
        bar.append((t_arrive, time.time()))
    st = check(xg, ctx)
    allbar = ctx.all_gather_object(bar)
    allp = ctx.all_gather_object(p.cpu().tolist())
    alll = ctx.all_gather_object(loss.cpu().tolist())
    if ctx.rank == 0:
        with open(out_path, "w") as f:
            json.dump({"status": st, "barrier": allbar, "params": allp, "losses": alll, "step_counter": int(sc.item())}, f)
    ctx.barrier()
    del xg
    shutdown(ctx)


if __name__ == "__main__":
    main()
