#!/usr/bin/env python3
"""Launch + synchronize floor of the HIP runtime as torch drives it, next to the bound weather
launch: is the driver's 20-step window bound by our kernel or by the runtime's completion wait?
`--spin` sets hipDeviceScheduleSpin before the device is initialised (host spins on the
completion signal instead of sleeping on an interrupt)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    spin = "--spin" in sys.argv
    if spin:
        import importlib.util
        tl = os.path.join(os.path.dirname(importlib.util.find_spec("torch").origin), "lib", "libamdhip64.so")
        hip = ctypes.CDLL(tl)
        print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)
    import torch

    import dct_amd  # noqa: F401
    from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params

    def best(fn, n=300):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e6, ts[0] * 1e6

    dev = torch.device("cuda", 0)
    # --dims 5,128,128,2 (default: the headline 3x128; 5,64,2 = the reference model)
    dims = [5, 128, 128, 2]
    if "--dims" in sys.argv:
        dims = [int(x) for x in sys.argv[sys.argv.index("--dims") + 1].split(",")]
    P = mlp_num_params(dims)
    k = FusedMLPKernel(dims, bmax=4)
    p = torch.randn(P, device=dev) * 0.1
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    N = 1 << 16
    X = torch.randn(N, 5, device=dev)
    Y = torch.randint(0, 2, (N,), device=dev, dtype=torch.int32)
    idx = torch.randint(0, N, (N,), device=dev, dtype=torch.int32)
    loss = torch.zeros(N // 4, device=dev)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    bl = k.prepare_train(p, m, v, X, Y, idx, n_items=N, batch=4, lr=1e-3, loss_out=loss, step_counter=ctr)
    tiny = torch.zeros(1, device=dev)
    from dct_amd.ops._native import native

    nat = native()
    stream = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    out = {
        "sync_only": best(torch.cuda.synchronize),
        "tiny_launch_sync": best(lambda: (tiny.add_(1.0), torch.cuda.synchronize())),
        "tiny_launch_stream_sync": best(lambda: (tiny.add_(1.0), torch.cuda.current_stream().synchronize())),
        # a one-thread native kernel through the same pybind + hipLaunchKernelGGL path: the floor
        # the weather launch's own prologue / epilogue sit on top of
        "native_null_launch_sync": best(lambda: (nat.zero_f32(tiny.data_ptr(), 1, stream), torch.cuda.synchronize())),
        "bound_s1_launch_sync": best(lambda: (bl.run(0, 1), torch.cuda.synchronize())),
        "bound_s20_launch_sync": best(lambda: (bl.run(0, 20), torch.cuda.synchronize())),
        "bound_s40_launch_sync": best(lambda: (bl.run(0, 40), torch.cuda.synchronize())),
    }
    tag = "spin" if spin else "env ROC_ACTIVE_WAIT_TIMEOUT=" + os.environ.get("ROC_ACTIVE_WAIT_TIMEOUT", "-")
    for name, (med, lo) in out.items():
        print(f"[{tag}] {name:26s} median {med:8.2f} us   min {lo:8.2f} us", flush=True)
    s1, s20, s40 = (out[f"bound_s{k}_launch_sync"][0] for k in (1, 20, 40))
    per = (s40 - s20) / 20.0
    print(f"dims {dims}: per step {per:.3f} us, fixed per launch+sync {s20 - 20 * per:.2f} us "
          f"(null launch+sync {out['native_null_launch_sync'][0]:.2f} us)", flush=True)


if __name__ == "__main__":
    main()
