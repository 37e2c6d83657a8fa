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
def test_hip_fit_with_graph_capture(cuda):
    from dct_amd.trainer import Trainer

    torch.manual_seed(0)
    X, Y = _data(2048, 32)
    ds = TensorDataset(X, Y)
    tl = DataLoader(torch.utils.data.Subset(ds, range(1792)), batch_size=128, shuffle=True)
    vl = DataLoader(torch.utils.data.Subset(ds, range(1792, 2048)), batch_size=128)
    m = TabTransformer(num_features=32, d_model=64, heads=4, layers=2, lr=3e-3)
    tr = Trainer(max_epochs=4, accelerator="gpu", engine="autograd", verbose=False, num_sanity_val_steps=0)
    tr.fit(m, tl, vl)
    assert tr.engine.graph_used
    assert tr.callback_metrics["val_acc"] > 0.75
