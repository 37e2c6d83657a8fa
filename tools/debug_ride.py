#!/usr/bin/env python3
"""Debug: the tabular executor step with Adam riding in the dW launches vs one Adam launch, graph
and eager, at B = 1024: per-layer max |dp| after each of 3 steps against the DCT_DW_INTO_ADAM=0 run."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

from test_graph_engine_gpu import _data, _engine  # noqa: E402


def run(into, ride, graph, B, steps=3):
    os.environ["DCT_DW_INTO_ADAM"] = into
    dims = [256, 1024, 1024, 1024, 2]
    X, Y = _data(8 * B, dims[0], seed=5)
    rows = torch.arange(X.shape[0])
    model, eng = _engine(dims, B, loss="ce", lr=1e-3, use_graph=graph)
    if ride is not None:
        eng.exe.adam_ride = ride
    eng.attach_data(X, Y, rows, rows[:B])
    n = eng.upload_epoch_indices(0, shuffle=False)
    loss = torch.zeros(16, device="cuda")
    snaps = []
    p_init = eng.p.cpu().clone()
    for s in range(steps):
        eng.run_steps(n, 1, loss, first_step=s)
        torch.cuda.synchronize()
        snaps.append(eng.p.cpu().clone())
        if s == 0:
            eng._mv0 = (p_init, eng.m.cpu().clone(), eng.v.cpu().clone(), eng.p.cpu().clone())
    return snaps, loss[:steps].cpu(), eng


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    ref, lref, eng = run("0", None, False, B)
    dims = [256, 1024, 1024, 1024, 2]
    offs = [0]
    for i in range(len(dims) - 1):
        offs.append(offs[-1] + dims[i] * dims[i + 1])
        offs.append(offs[-1] + dims[i + 1])
    print("ref losses", lref.tolist(), "P", eng.P, "offsets", offs)
    for into, ride, graph in (("1", False, False), ("1", True, False), ("1", False, True), ("1", True, True)):
        snaps, l, e = run(into, ride, graph, B)
        print(f"into={into} ride={ride} graph={graph} losses={l.tolist()} partial_layers={e.exe.partial_layers}")
        p0, m1, v1, pr = e._mv0
        _, m0, v0, pq = eng._mv0
        lo = offs[4]
        for j in (lo, lo + 1, lo + 5, lo + 1000, lo + 100000):
            print(f"   W2[{j - lo}] p_init {float(p0[j]):+.5e} p_ref {float(pq[j]):+.5e} p {float(pr[j]):+.5e} "
                  f"m_ref {float(m0[j]):+.3e} m {float(m1[j]):+.3e} v_ref {float(v0[j]):.3e} v {float(v1[j]):.3e}")
        for nm, a_, b_ in (("W1", offs[2], offs[3]), ("W2", offs[4], offs[5])):
            dd = (pr[a_:b_] - pq[a_:b_]).abs()
            bad = torch.nonzero(dd > 1e-5).flatten()
            print(f"   {nm}: {bad.numel()} bad of {b_ - a_}; first {bad[:12].tolist()} last {bad[-4:].tolist()}")
            if bad.numel():
                j = bad[:6] + a_
                ratio = (pr[j] - p0[j]) / (pq[j] - p0[j])
                print(f"      ratio upd/ref {ratio.tolist()}  m {m1[j].tolist()} v {v1[j].tolist()}")
                blk = (bad // 4) // 512
                print(f"      distinct 512-thread blocks (rel. range start): {torch.unique(blk)[:20].tolist()} n={torch.unique(blk).numel()}")
        dm = (m1 - m0).abs()
        print("   step0 max|dm| per range " + " ".join(f"{float(dm[offs[i]:offs[i + 1]].max()):.1e}" for i in range(len(offs) - 1)))
        for s, (a, b) in enumerate(zip(snaps, ref)):
            d = (a - b).abs()
            per = [float(d[offs[i]:offs[i + 1]].max()) if offs[i + 1] > offs[i] else 0.0 for i in range(len(offs) - 1)]
            print(f"   step {s}: max|dp| per W/b range " + " ".join(f"{x:.1e}" for x in per))


if __name__ == "__main__":
    main()
