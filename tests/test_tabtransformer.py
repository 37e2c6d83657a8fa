"""TabTransformer (BASELINE config 5): CPU reference path, and the HIP path (ops/nn.py) against it."""
import pytest
import torch
from torch.utils.data import DataLoader, TensorDataset

import dct_amd  # noqa: F401
from dct_amd.models import build_model
from dct_amd.models.tabtransformer import TabTransformer


def _data(n=512, f=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, f, generator=g)
    Y = ((X[:, : f // 2].sum(1) - X[:, f // 2:].sum(1)) > 0).long()
    return X, Y


def test_cpu_forward_backward_and_registry():
    m = build_model("tabtransformer", 16, d_model=32, heads=4, layers=2)
    assert isinstance(m, TabTransformer) and m.hparams["num_features"] == 16
    X, Y = _data(8)
    out = m(X)
    assert out.shape == (8, 2)
    loss = torch.nn.functional.cross_entropy(out, Y)
    loss.backward()
    assert all(p.grad is not None for p in m.parameters())


def test_cpu_fit_learns(tmp_path):
    from dct_amd.trainer import Trainer

    torch.manual_seed(0)
    X, Y = _data(1024)
    ds = TensorDataset(X, Y)
    tl = DataLoader(torch.utils.data.Subset(ds, range(800)), batch_size=32, shuffle=True)
    vl = DataLoader(torch.utils.data.Subset(ds, range(800, 1024)), batch_size=64)
    m = TabTransformer(num_features=16, d_model=32, heads=4, layers=2, lr=3e-3)
    tr = Trainer(max_epochs=4, accelerator="cpu", engine="autograd", verbose=False, num_sanity_val_steps=0)
    tr.fit(m, tl, vl)
    assert tr.callback_metrics["val_acc"] > 0.75


@pytest.mark.gpu
@pytest.mark.parametrize("F_", [32, 64])  # 64 features = the whole-block fused kernel shape
def test_hip_path_matches_torch_reference(cuda, F_):
    torch.manual_seed(1)
    B = 64
    ref = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2)
    hip = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2)
    hip.load_state_dict(ref.state_dict())
    hip.to(cuda)
    X, Y = _data(B, F_)
    lr_ = torch.nn.functional.cross_entropy(ref(X), Y)
    lr_.backward()
    lh = torch.nn.functional.cross_entropy(hip(X.to(cuda)), Y.to(cuda))
    lh.backward()
    torch.cuda.synchronize()
    assert abs(lh.item() - lr_.item()) < 2e-2
    for (n, pr), (_, ph) in zip(ref.named_parameters(), hip.named_parameters()):
        rel = (ph.grad.cpu() - pr.grad).norm() / (pr.grad.norm() + 1e-12)
        assert rel < 0.1, (n, float(rel))


@pytest.mark.gpu
@pytest.mark.parametrize("F_,min_acc", [(32, 0.75), (64, 0.6)])  # 64: fused kernels; the CPU path reaches 0.64 there
def test_hip_fit_with_graph_capture(cuda, F_, min_acc):
    from dct_amd.trainer import Trainer

    torch.manual_seed(0)
    X, Y = _data(2048, F_)
    ds = TensorDataset(X, Y)
    tl = DataLoader(torch.utils.data.Subset(ds, range(1792)), batch_size=128, shuffle=True)
    vl = DataLoader(torch.utils.data.Subset(ds, range(1792, 2048)), batch_size=128)
    m = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2, lr=3e-3)
    tr = Trainer(max_epochs=4, accelerator="gpu", engine="autograd", verbose=False, num_sanity_val_steps=0)
    tr.fit(m, tl, vl)
    assert tr.engine.graph_used
    assert tr.callback_metrics["val_acc"] > min_acc


@pytest.mark.gpu
@pytest.mark.parametrize("F_", [32, 64])
def test_device_loop_matches_host_loop(cuda, F_):
    """AutogradEngine.run_device_steps (one captured graph per step: device batch gather, counter,
    grad zeroing, loss record and cursor in the Adam epilogue) trains exactly like train_step; at 64
    features the gather / counter / zeroing ride in the first fused block's launch (ops/nn.py
    fold_batch_gather)."""
    from dct_amd.parallel.dist import init_distributed
    from dct_amd.trainer.engines import AutogradEngine
    from dct_amd.trainer.trainer import seed_everything

    ctx = init_distributed("gpu")
    X, Y = _data(4096, F_, seed=3)
    rows = torch.randperm(4096, generator=torch.Generator().manual_seed(1))
    B, steps = 128, 12
    res = []
    for device_loop in (False, False, True):
        seed_everything(7)
        m = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2, lr=3e-3)
        eng = AutogradEngine(m, ctx, B, seed=7)
        eng.attach_data(X.to(cuda), Y.to(cuda), rows[:3584], rows[3584:])
        rows_dev = eng.train_rows.to(cuda)
        loss = torch.zeros(steps, device=cuda)
        if device_loop:
            eng.run_device_steps(rows_dev, 0, 5, loss)        # warm-up + capture + replays
            eng.run_device_steps(rows_dev, 5, steps - 5, loss)  # resumes at the device cursor
        else:
            for s in range(steps):
                loss[s] = eng.train_step(rows_dev[s * B:(s + 1) * B], s)
        torch.cuda.synchronize()
        res.append((loss.cpu(), eng.flat_p.detach().cpu().clone(), eng.optimizer.step_count))
        if device_loop:
            assert eng.graph_used
            # 64 features: the first fused block gathers the batch itself (no prologue launch)
            assert eng.gather_folded == (F_ == 64), eng.gather_folded
    (l0, p0, c0), (lh, ph, _), (l1, p1, c1) = res
    assert c0 == c1 == steps
    assert torch.isfinite(l1).all() and (l1 != 0).all()
    assert torch.allclose(l0, l1, rtol=2e-3, atol=2e-4), (l0, l1)
    # split-K atomics make two identical host-loop runs differ slightly (Adam turns near-zero
    # gradient noise into +-lr steps); the device loop must sit within that run-to-run spread
    noise = float((p0 - ph).norm() / p0.norm())
    diff = float((p0 - p1).norm() / p0.norm())
    assert diff < max(3 * noise, 1e-4), (diff, noise)


@pytest.mark.gpu
def test_deferred_dw_matches_in_stream(cuda, monkeypatch):
    """Fused-block dW GEMMs deferred to one grouped launch after backward (DCT_TT_DW_DEFER=1) train
    the same trajectory as the per-block launches on the compute stream, eager steps and captured
    step graphs alike."""
    knob = "DCT_TT_DW_DEFER"
    from dct_amd.parallel.dist import init_distributed
    from dct_amd.trainer.engines import AutogradEngine
    from dct_amd.trainer.trainer import seed_everything

    ctx = init_distributed("gpu")
    F_ = 64
    X, Y = _data(4096, F_, seed=4)
    rows = torch.randperm(4096, generator=torch.Generator().manual_seed(2))
    B, steps = 128, 12
    res = {}
    for side in ("1", "0", "0"):
        monkeypatch.setenv(knob, side)
        seed_everything(7)
        m = TabTransformer(num_features=F_, d_model=64, heads=4, layers=3, lr=3e-3)
        eng = AutogradEngine(m, ctx, B, seed=7)
        eng.attach_data(X.to(cuda), Y.to(cuda), rows[:3584], rows[3584:])
        rows_dev = eng.train_rows.to(cuda)
        loss = torch.zeros(steps, device=cuda)
        eng.run_device_steps(rows_dev, 0, steps, loss)  # eager warm-up steps, capture, replays
        torch.cuda.synchronize()
        assert eng.graph_used
        res.setdefault(side, []).append((loss.cpu(), eng.flat_p.detach().cpu().clone()))
    (l1, p1), = res["1"]
    (l0, p0), (lh, ph) = res["0"]
    assert torch.isfinite(l1).all() and (l1 != 0).all()
    assert torch.allclose(l0, l1, rtol=2e-3, atol=2e-4), (l0, l1)
    noise = float((p0 - ph).norm() / p0.norm())
    diff = float((p0 - p1).norm() / p0.norm())
    assert diff < max(3 * noise, 1e-4), (diff, noise)


@pytest.mark.gpu
def test_fused_embedding_matches_separate_kernel(cuda, monkeypatch):
    """The first block embedding the features itself (models/tabtransformer.py FUSED_EMBED, tt_block
    embed=(E, c)) gives the same loss bit for bit (same fmaf per element as tt_io.hip's embed kernel)
    and the same gradients as the separate embedding kernel writing the block input; the pooled head
    and the fused backward on both sides."""
    from dct_amd.models import tabtransformer as ttm

    torch.manual_seed(5)
    F_, B = 64, 256
    base = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2)
    X, Y = _data(B, F_, seed=6)
    X, Y = X.to(cuda), Y.to(cuda)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(ttm, "FUSED_EMBED", fused)
        m = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2)
        m.load_state_dict(base.state_dict())
        m.to(cuda)
        loss = m.training_step((X, Y), 0)
        loss = loss["loss"] if isinstance(loss, dict) else loss
        loss.backward()
        torch.cuda.synchronize()
        res[fused] = (loss.detach().cpu(), {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()})
    (l1, g1), (l0, g0) = res[True], res[False]
    assert torch.equal(l1, l0), (l1, l0)
    for n in g0:
        rel = float((g1[n] - g0[n]).norm() / (g0[n].norm() + 1e-12))
        assert rel < 1e-4, (n, rel)


@pytest.mark.gpu
def test_training_step_fused_head_matches_two_launch_head(cuda):
    """training_step under unit_loss_seed() (the autograd engine's step: backward seed exactly 1) runs
    the pooled classifier head's backward inside its forward launch (csrc/tt_io.hip dct_tt_head_fused):
    the loss bit for bit and every parameter gradient (to float-atomic rounding) equal the head's
    forward + backward launches."""
    from dct_amd.ops.nn import unit_loss_seed

    torch.manual_seed(3)
    B, F_ = 128, 64
    X, Y = _data(B, F_)
    X, Y = X.to(cuda), Y.to(cuda)
    res = {}
    for fused in (False, True):
        torch.manual_seed(4)
        m = TabTransformer(num_features=F_, d_model=64, heads=4, layers=2).to(cuda)
        m.train()
        if fused:
            with unit_loss_seed():
                loss = m.training_step((X, Y), 0)
                loss.backward(torch.ones_like(loss))
        else:
            loss = m.training_step((X, Y), 0)
            loss.backward(torch.ones_like(loss))
        torch.cuda.synchronize()
        res[fused] = (float(loss), {n: p.grad.detach().clone() for n, p in m.named_parameters()})
    (l0, g0), (l1, g1) = res[False], res[True]
    assert l0 == l1, (l0, l1)
    for n in g0:
        rel = (g1[n] - g0[n]).norm() / (g0[n].norm() + 1e-12)
        assert rel < 1e-5, (n, float(rel))
