"""The bf16 MFMA GEMM on the tabular MLP step's own shapes (interleaved rounds, one process).

    python tools/bench_gemm_mlp.py [--rounds 5]

Shapes (batch 4096, 256-1024-1024-1024-2, bench.py --model tabular-mlp-4x1024):
  forward  Y = X W^T      4096x1024x256 (NT), 4096x1024x1024 (NT) x2
  dX       dZ W           4096x1024x1024 (NN) x2, bf16 out
  dW       dZ^T X         1024x1024x4096 (TN, fp32 split-K) x2, 1024x256x4096
plus the TabTransformer step's projection / FFN shapes (32768 token rows, d 64, ffn 256).
Prints one JSON line per shape with the median over rounds, next to hipBLASLt on the same operands.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops._native import native  # noqa: E402

SHAPES = [  # name, M, N, K, ta, tb, out_f32
    ("fwd_l0", 4096, 1024, 256, 0, 1, 0),
    ("fwd_l1", 4096, 1024, 1024, 0, 1, 0),
    ("dx_l1", 4096, 1024, 1024, 0, 0, 0),
    ("dw_l1", 1024, 1024, 4096, 1, 0, 1),
    ("dw_l0", 1024, 256, 4096, 1, 0, 1),
    # TabTransformer (batch 512 x 64 tokens = 32768 rows, d 64, ffn 256)
    ("tt_fwd_qkv", 32768, 192, 64, 0, 1, 0),
    ("tt_fwd_fc1", 32768, 256, 64, 0, 1, 0),
    ("tt_fwd_fc2", 32768, 64, 256, 0, 1, 0),
    ("tt_dx_fc1", 32768, 64, 256, 0, 0, 0),
    ("tt_dx_fc2", 32768, 256, 64, 0, 0, 0),
    ("tt_dw_qkv", 192, 64, 32768, 1, 0, 1),
    ("tt_dw_fc1", 256, 64, 32768, 1, 0, 1),
    ("tt_dw_fc2", 64, 256, 32768, 1, 0, 1),
    ("tt_dw_o", 64, 64, 32768, 1, 0, 1),
]
if os.environ.get("AB_SET") == "layout":  # transformer dW shapes in every operand layout (what would a
    # feature-major copy of the activations buy?): (1,0) = today's dZ^T X on token-major storage
    SHAPES = [(f"{n}_ta{ta}tb{tb}", M, N, K, ta, tb, 1) for n, M, N, K, *_ in SHAPES if n.startswith("tt_dw")
              for ta, tb in ((1, 0), (0, 1), (0, 0), (1, 1))]
if os.environ.get("AB_SET") == "dwcmp":  # the tabular dW shapes: default launch vs hipBLASLt
    SHAPES = [s for s in SHAPES if s[0] in ("dw_l1", "dw_l0", "fwd_l1", "dx_l1")]
# (round 1-4 A/B variants - pipeline depths, split-K targets, tile heights, in-launch split-K - were
# deleted with their knobs in round 5; their results are in profiles/gemm_*_r*.log)
VARIANTS = {"default": {}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--sets", type=int, default=1,
                    help="operand sets rotated per launch: > 3 sets of the 4096x1024 shapes exceed the 8 XCDs' L2 "
                         "(the in-step situation: operands from the Infinity Cache, not a hot L2)")
    a = ap.parse_args()
    nat = native()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    res = {}
    bufs = {}
    for name, M, N, K, ta, tb, of in SHAPES:
        sets = []
        for _ in range(a.sets):
            A = (torch.rand(K, M, device=dev) * 2 - 1 if ta else torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            B = (torch.rand(N, K, device=dev) * 2 - 1 if tb else torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)
            sets.append((A, B))
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if of else torch.bfloat16)
        bufs[name] = (sets, C)
    for _ in range(a.rounds):
        for vname, env in VARIANTS.items():
            for name, M, N, K, ta, tb, of in SHAPES:
                sets, C = bufs[name]
                cyc = [0]

                def run():
                    A, B = sets[cyc[0] % len(sets)]
                    cyc[0] += 1
                    nat.gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), 0, M, N, K, A.stride(0), B.stride(0), N,
                                  ta, tb, 0, of, 0, 0, st)
                for _ in range(3):
                    run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    run()
                e.record()
                torch.cuda.synchronize()
                res.setdefault((name, vname), []).append(s.elapsed_time(e) / a.iters * 1e3)
    for name, M, N, K, ta, tb, of in SHAPES:  # hipBLASLt (torch.matmul) on the same operands
        (A, B), C = bufs[name][0][0], bufs[name][1]
        At = A.t() if ta else A
        Bt = B.t() if tb else B
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(At, Bt, out=out)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            torch.matmul(At, Bt, out=out)
        e.record()
        torch.cuda.synchronize()
        res[(name, "hipblaslt")] = [s.elapsed_time(e) / a.iters * 1e3]
    for (name, vname), ts in res.items():
        M, N, K = next((m, n, k) for nm, m, n, k, *_ in SHAPES if nm == name)
        us = statistics.median(ts)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": vname, "us_median": round(us, 2),
                          "us_min": round(min(ts), 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
