"""Wide-MLP graph-captured step (csrc/mlp_executor.cpp + trainer/graph_engine.py) against a
plain-torch fp32 reference of the same step (bf16 operands -> bf16-level tolerances)."""
import math

import pytest
import torch
import torch.nn.functional as F

import dct_amd  # noqa: F401
from dct_amd.models.mlp import MLPClassifier
from dct_amd.parallel.dist import init_distributed
from dct_amd.trainer.engines import adam_hparams_from
from dct_amd.trainer.graph_engine import GraphMLPEngine

pytestmark = pytest.mark.gpu


def _data(n, d, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    w = torch.randn(d, generator=g)
    Y = ((X @ w) > 0).long()
    return X, Y


def _engine(dims, B, loss="mse", lr=1e-3, use_graph=True):
    torch.manual_seed(0)
    model = MLPClassifier(dims[0], hidden=tuple(dims[1:-1]), num_classes=dims[-1], dropout=0.0, loss=loss, lr=lr)
    ctx = init_distributed("gpu")
    eng = GraphMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()),
                         use_graph=use_graph)
    return model, eng


@pytest.mark.parametrize("loss", ["mse", "ce"])
@pytest.mark.parametrize("dims,B", [([64, 256, 256, 2], 64), ([256, 1024, 1024, 1024, 2], 256), ([32, 96, 3], 50)])
def test_one_step_gradients_match_torch(dims, B, loss, cuda):
    """lr = 0: one executor step leaves the weights and exposes g = dL/dp; compare with autograd
    on the same bf16-rounded inputs and weights."""
    model, eng = _engine(dims, B, loss=loss, lr=0.0)
    X, Y = _data(4 * B, dims[0])
    Y = Y % dims[-1]
    rows = torch.arange(4 * B)
    eng.attach_data(X, Y, rows, rows[:B])
    eng.idx[:B].copy_(torch.arange(B, dtype=torch.int32))
    loss_out = torch.zeros(1, device=cuda)
    eng.cursor.zero_()
    eng._step(B, loss_out, B)
    torch.cuda.synchronize()
    # reference: fp32 autograd on bf16-rounded data/weights
    ref = MLPClassifier(dims[0], hidden=tuple(dims[1:-1]), num_classes=dims[-1], dropout=0.0, loss=loss)
    with torch.no_grad():
        for (n, t), (_, t0) in zip(ref.state_dict().items(), model.state_dict().items()):
            t.copy_(t0.to(torch.bfloat16).float() if "weight" in n else t0)
    xb = X[:B].to(torch.bfloat16).float()
    # forward values rounded to bf16 after every layer like the kernels' bf16 activations
    # (straight-through: the rounding does not enter the gradient)
    h = xb
    for mod in ref.net:
        h = mod(h)
        if isinstance(mod, torch.nn.Linear):
            h = h + (h.to(torch.bfloat16).float() - h).detach()
    logits = h
    if loss == "ce":
        lref = F.cross_entropy(logits, Y[:B])
    else:
        lref = F.mse_loss(logits, F.one_hot(Y[:B], dims[-1]).float())
    lref.backward()
    want = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    got = eng.g[: eng.P].cpu()
    rel = (got - want).norm() / want.norm()
    assert rel < 4e-2, rel
    assert abs(float(loss_out.item()) - lref.item()) < 2e-2 * max(1.0, abs(lref.item()))
    assert int(eng.cursor.item()) == 1 and int(eng.step_counter.item()) == 1


def test_graph_replay_equals_eager_and_learns(cuda):
    dims, B = [64, 256, 256, 2], 128
    X, Y = _data(40 * B + 37, dims[0], seed=3)
    n = X.shape[0]
    res = []
    for use_graph in (True, False):
        model, eng = _engine(dims, B, lr=1e-3, use_graph=use_graph)
        rows = torch.arange(n)
        eng.attach_data(X, Y, rows[: 40 * B + 37], rows[:512])
        losses = []
        for ep in range(3):
            losses.append(eng.train_epoch(ep).cpu())
        torch.cuda.synchronize()
        assert eng.graph_used == use_graph
        res.append((torch.cat(losses), eng.p.cpu(), eng))
    (l_g, p_g, eg), (l_e, p_e, _) = res
    assert l_g.numel() == 3 * math.ceil((40 * B + 37) / B)
    # bias grads and split-K dW use float atomics: runs agree to rounding, not bit for bit (and
    # Adam turns rounding noise on ~0 gradients into +-lr steps), so compare in norm
    assert torch.allclose(l_g, l_e, atol=1e-3), (l_g - l_e).abs().max()
    assert (p_g - p_e).norm() / p_e.norm() < 1e-2
    assert l_g[-10:].mean() < l_g[:10].mean()
    vl, va = eg.validate()
    assert va > 0.7


def test_trainer_fit_graph_engine_writes_checkpoint(tmp_path, cuda):
    from torch.utils.data import DataLoader, TensorDataset

    from dct_amd.ckpt import ModelCheckpoint, load_checkpoint
    from dct_amd.trainer import Trainer

    X, Y = _data(3000, 64, seed=1)
    ds = TensorDataset(X, Y)
    tl = DataLoader(torch.utils.data.Subset(ds, range(2400)), batch_size=256, shuffle=True)
    vl = DataLoader(torch.utils.data.Subset(ds, range(2400, 3000)), batch_size=256)
    model = MLPClassifier(64, hidden=(128, 128), dropout=0.0, loss="mse", lr=1e-3)
    ck = ModelCheckpoint(dirpath=str(tmp_path), filename="best-{epoch:02d}", monitor="val_loss", mode="min",
                         save_top_k=1, save_last=True)
    tr = Trainer(max_epochs=2, accelerator="gpu", callbacks=[ck], engine="graph", verbose=False)
    tr.fit(model, tl, vl)
    assert tr.engine.name == "graph"
    sd = load_checkpoint(str(tmp_path / "last.ckpt"))["state_dict"]
    assert set(sd) == set(model.state_dict())
    assert tr.callback_metrics["val_loss"] < 0.5


@pytest.mark.parametrize("B,extra", [(1024, 0), (4096, 0), (1024, 300)])
def test_dw_slices_into_adam_match_reduce_path(B, extra, cuda, monkeypatch):
    """Without a DDP reducer the executor hands the split-K dW slices of the 1024x1024 hidden
    layers (2-4 slices) and of the 256-wide input layer (8 slices at B = 4096, fp32 atomics into g
    otherwise) to Adam, summed there in slice order: the same trajectory as DCT_DW_INTO_ADAM=0.
    ``extra`` rows make every epoch end with a partial batch: its dW falls back to g
    for that step and the trajectories still agree."""
    dims = [256, 1024, 1024, 1024, 2]
    X, Y = _data(8 * B + extra, dims[0], seed=5)
    rows = torch.arange(X.shape[0])
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DCT_DW_INTO_ADAM", mode)
        model, eng = _engine(dims, B, loss="ce", lr=1e-3)
        eng.attach_data(X, Y, rows, rows[:B])
        losses = torch.cat([eng.train_epoch(ep).cpu() for ep in range(2)])
        torch.cuda.synchronize()
        res[mode] = (losses, eng.p.cpu())
        if mode == "1":
            assert eng.exe.partial_layers == 3
            assert (eng.exe.part_fallbacks > 0) == (extra > 0), eng.exe.part_fallbacks
    (l1, p1), (l0, p0) = res["1"], res["0"]
    assert torch.isfinite(l1).all()
    assert torch.allclose(l1, l0, atol=1e-3), (l1 - l0).abs().max()
    assert (p1 - p0).norm() / p0.norm() < 1e-2


@pytest.mark.parametrize("extra", [0, 300])
def test_adam_riding_in_dw_launches_matches_one_adam_launch(extra, cuda):
    """Without a DDP reducer the executor runs each layer's Adam in extra workgroups of the next
    lower layer's dW launch (csrc/gemm_bf16.hip gemm2_dw_adam_kernel) and only the input layer's in
    the final launch: the same trajectory as one Adam launch at the end of the step (the bias
    gradients' float atomics make runs agree to rounding, not bit for bit).  ``extra``: partial last
    batches take the one-launch path."""
    dims, B = [256, 1024, 1024, 1024, 2], 4096
    X, Y = _data(6 * B + extra, dims[0], seed=7)
    rows = torch.arange(X.shape[0])
    res = {}
    for ride in (True, False):
        model, eng = _engine(dims, B, loss="mse", lr=1e-3, use_graph=False)
        eng.exe.adam_ride = ride
        eng.attach_data(X, Y, rows, rows[:B])
        losses = torch.cat([eng.train_epoch(ep).cpu() for ep in range(2)])
        torch.cuda.synchronize()
        assert eng.exe.adam_ride == ride and eng.exe.partial_layers == 3
        res[ride] = (losses, eng.p.cpu(), eng.m.cpu(), eng.v.cpu(), int(eng.step_counter.item()))
    (l1, p1, m1, v1, s1), (l0, p0, m0, v0, s0) = res[True], res[False]
    assert s1 == s0
    assert torch.isfinite(l1).all() and torch.allclose(l1, l0, atol=1e-4), (l1 - l0).abs().max()
    assert (p1 - p0).norm() / p0.norm() < 1e-3
    assert (m1 - m0).norm() / m0.norm() < 1e-2 and (v1 - v0).norm() / v0.norm() < 1e-2


@pytest.mark.parametrize("extra", [0, 300])
def test_gather_fused_into_first_forward_gemm_matches_gather_launch(extra, cuda):
    """Full batches gather their rows inside the first forward GEMM (csrc/gemm_bf16.hip
    dct_gemm_bf16_gather_fwd: dataset rows straight into the LDS A images, the gathered rows written
    out for the dW GEMM, labels / step counter / gradient clearing riding along) instead of the gather
    launch: the same trajectory as the gather launch (float-atomic bias gradients: equal to rounding).
    ``extra``: the partial last batch of each epoch takes the gather launch."""
    dims, B = [256, 1024, 1024, 1024, 2], 4096
    X, Y = _data(6 * B + extra, dims[0], seed=9)
    rows = torch.arange(X.shape[0])
    res = {}
    for fuse in (True, False):
        model, eng = _engine(dims, B, loss="ce", lr=1e-3, use_graph=False)  # (eager: one host step per step)
        eng.exe.set_gather_fuse(fuse)
        eng.attach_data(X, Y, rows, rows[:B])
        losses = torch.cat([eng.train_epoch(ep).cpu() for ep in range(2)])
        torch.cuda.synchronize()
        full = 2 * (X.shape[0] // B)
        assert eng.exe.gather_fused_steps == (full if fuse else 0), eng.exe.gather_fused_steps
        res[fuse] = (losses, eng.p.cpu(), eng.m.cpu(), int(eng.step_counter.item()))
    (l1, p1, m1, s1), (l0, p0, m0, s0) = res[True], res[False]
    assert s1 == s0 == 2 * -(-X.shape[0] // B)
    assert torch.isfinite(l1).all() and torch.allclose(l1, l0, atol=1e-4), (l1 - l0).abs().max()
    assert (p1 - p0).norm() / p0.norm() < 1e-3
    assert (m1 - m0).norm() / m0.norm() < 1e-2

