"""Numerics of the HIP kernels against plain-torch fp32 references (run on a real MI355X)."""
import math

import pytest
import torch
import torch.nn.functional as F

import dct_amd  # noqa: F401
from dct_amd.ops._native import native
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params, reference_mlp_forward

pytestmark = pytest.mark.gpu


def _ref_net(dims):
    layers = []
    for i in range(len(dims) - 1):
        layers.append(torch.nn.Linear(dims[i], dims[i + 1]))
        if i < len(dims) - 2:
            layers.append(torch.nn.ReLU())
    return torch.nn.Sequential(*layers)


def _flat(net):
    return torch.cat([t.detach().reshape(-1) for t in net.state_dict().values()])


def _ref_loss(logits, y, kind):
    if kind == "ce":
        return F.cross_entropy(logits, y)
    return F.mse_loss(logits, F.one_hot(y, logits.shape[1]).float())


# DCT_MLP_BLOCK setting of a kernel variant name: "lds-<variant>" selects one of the 3x128 trainers
# (default = mlp_block5 for the exact weather shape D0 <= 8 -> 128 -> 128 -> 2 and 8-wave
# mlp_block3 for every other 3x128 shape, b3 = mlp_block3 everywhere, noblock = the generic LDS
# trainer)
_VARIANTS = {"": "-1", "noblock": "0", "b3": "3"}


def _set_kernel_env(monkeypatch, kernel):
    parts = kernel.split("-")
    monkeypatch.setenv("DCT_MLP_KERNEL", parts[0])
    monkeypatch.setenv("DCT_MLP_BLOCK", _VARIANTS[parts[1] if len(parts) > 1 else ""])


@pytest.fixture(autouse=True)
def _fresh_knobs():
    """The native launchers read their DCT_* knobs at plan / bind time (csrc/knobs.h): start every
    test from the environment as it is now (a previous test's monkeypatch is undone by then)."""
    native().reload_knobs()


def setknob(monkeypatch, name, value=None):
    """Set (or, with value None, clear) one DCT_* knob and re-read the native knob struct."""
    if value is None:
        monkeypatch.delenv(name, raising=False)
    else:
        monkeypatch.setenv(name, value)
    native().reload_knobs()


def test_native_loaded_and_arch():
    nat = native()
    assert nat.device_count() >= 1
    assert "gfx950" in nat.arch_name(0)


KERNELS = ["auto", "lds", "lds-noblock", "lds-b3"]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("loss", ["ce", "mse"])
@pytest.mark.parametrize("dims,B", [([5, 64, 2], 4), ([5, 128, 128, 2], 4), ([5, 64, 2], 3), ([9, 48, 64, 3], 4),
                                    ([16, 32, 48, 32, 3], 16), ([5, 128, 128, 2], 16), ([7, 20, 2], 9),
                                    ([7, 20, 2], 8), ([12, 40, 4], 6), ([16, 64, 3], 2), ([5, 64, 2], 1),
                                    # mlp_block5 below its full batch and at its input-width bounds
                                    ([3, 128, 128, 2], 3), ([8, 128, 128, 2], 1), ([1, 128, 128, 2], 2),
                                    # mlp_block5 with two micro-batches per step (batch 5..8)
                                    ([5, 128, 128, 2], 8), ([8, 128, 128, 2], 5), ([3, 128, 128, 2], 7),
                                    ([5, 128, 128, 2], 6)])
def test_fused_train_matches_torch_adam(dims, B, loss, kernel, cuda, monkeypatch):
    _set_kernel_env(monkeypatch, kernel)
    torch.manual_seed(1)
    N, n_items = 301, 50
    X = torch.randn(N, dims[0])
    Y = torch.randint(0, dims[-1], (N,))
    idx = torch.randperm(N)[:n_items]
    net = _ref_net(dims)
    p = _flat(net).to(cuda)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    steps = math.ceil(n_items / B)
    losses = torch.zeros(steps, device=cuda)
    k = FusedMLPKernel(dims, bmax=4 if B <= 4 else 16)
    k.train(p, m, v, X.to(cuda), Y.to(cuda, torch.int32), idx.to(cuda, torch.int32), n_items=n_items, batch=B,
            steps=steps, t0=0, lr=0.01, loss=loss, loss_out=losses)
    opt = torch.optim.Adam(net.parameters(), lr=0.01)
    ref_losses = []
    for s in range(steps):
        rows = idx[s * B:(s + 1) * B]
        opt.zero_grad()
        l = _ref_loss(net(X[rows]), Y[rows], loss)
        l.backward()
        opt.step()
        ref_losses.append(l.item())
    got = p.cpu()
    want = _flat(net)
    err = (got - want).abs()
    assert err.median() < 1e-5, err.median()
    assert err.max() < 2e-3, err.max()
    assert torch.allclose(losses.cpu(), torch.tensor(ref_losses), atol=2e-4, rtol=1e-3)
    # moments written back in torch flat order
    st = opt.state_dict()["state"]
    ref_m = torch.cat([st[i]["exp_avg"].reshape(-1) for i in range(len(st))])
    assert torch.allclose(m.cpu(), ref_m, atol=1e-4, rtol=1e-2)


@pytest.mark.parametrize("kernel", ["auto", "lds-b3"])
@pytest.mark.parametrize("loss", ["ce", "mse"])
def test_weather_3x128_weight_decay_matches_torch_adam(kernel, loss, cuda, monkeypatch):
    """The 3x128 trainers' L2 term (torch Adam weight_decay: g += wd * p) - mlp_block5's WD
    instantiation by default, mlp_block3's with lds-b3 - against torch.optim.Adam."""
    _set_kernel_env(monkeypatch, kernel)
    torch.manual_seed(6)
    dims, B, N, n_items = [5, 128, 128, 2], 4, 200, 60
    X = torch.randn(N, 5)
    Y = torch.randint(0, 2, (N,))
    idx = torch.randperm(N)[:n_items]
    net = _ref_net(dims)
    p = _flat(net).to(cuda)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    steps = n_items // B
    losses = torch.zeros(steps, device=cuda)
    k = FusedMLPKernel(dims, bmax=4)
    k.train(p, m, v, X.to(cuda), Y.to(cuda, torch.int32), idx.to(cuda, torch.int32), n_items=n_items, batch=B,
            steps=steps, t0=0, lr=0.01, weight_decay=0.05, loss=loss, loss_out=losses)
    opt = torch.optim.Adam(net.parameters(), lr=0.01, weight_decay=0.05)
    for s in range(steps):
        rows = idx[s * B:(s + 1) * B]
        opt.zero_grad()
        _ref_loss(net(X[rows]), Y[rows], loss).backward()
        opt.step()
    err = (p.cpu() - _flat(net)).abs()
    assert err.median() < 1e-5, err.median()
    assert err.max() < 2e-3, err.max()


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("dims,B", [([5, 64, 2], 4), ([5, 128, 128, 2], 4), ([12, 40, 40, 5], 13),
                                    ([9, 48, 64, 3], 4), ([20, 128, 128, 4], 3), ([32, 128, 128, 1], 4),
                                    ([8, 128, 128, 2], 3), ([2, 128, 128, 2], 1), ([5, 128, 128, 2], 8),
                                    ([7, 128, 128, 2], 6)])
def test_fused_grad_mode_matches_autograd(dims, B, kernel, cuda, monkeypatch):
    _set_kernel_env(monkeypatch, kernel)
    torch.manual_seed(2)
    N = 64
    X = torch.randn(N, dims[0])
    Y = torch.randint(0, dims[-1], (N,))
    idx = torch.arange(B, dtype=torch.int32)
    net = _ref_net(dims)
    p = _flat(net).to(cuda)
    P = mlp_num_params(dims)
    g = torch.zeros(P + 1, device=cuda)
    k = FusedMLPKernel(dims, bmax=4 if B <= 4 else 16)
    k.train(p, None, None, X.to(cuda), Y.to(cuda, torch.int32), idx.to(cuda), n_items=B, batch=B, steps=1, t0=0,
            lr=0.01, grad_out=g)
    l = F.cross_entropy(net(X[:B]), Y[:B]) if dims[-1] > 1 else F.cross_entropy(net(X[:B]), Y[:B] * 0)
    l.backward()
    want = torch.cat([q.grad.reshape(-1) for q in net.parameters()])
    assert torch.allclose(g[:P].cpu(), want, atol=1e-6, rtol=1e-4)
    assert abs(g[P].item() - l.item()) < 1e-5


@pytest.mark.parametrize("dims,B,n_items", [([5, 128, 128, 2], 4, 30), ([8, 128, 128, 2], 3, 13),
                                            ([1, 128, 128, 2], 2, 9)])
def test_block5_grad_mode_staged_batches(dims, B, n_items, cuda):
    """mlp_block5's grad mode at the device cursor (the DDP step path, one launch per step): each
    launch stages the next batch's x / label words in ``stage`` (tagged batch + 1) and the next
    launch reads them instead of gathering.  Every launch's gradients and loss must equal the
    unstaged launch of the same batch bit for bit - staged hits, the partial last batch, and a
    cursor jump (tag mismatch -> gather) included."""
    torch.manual_seed(6)
    N = 200
    X = torch.randn(N, dims[0]).to(cuda)
    Y = torch.randint(0, dims[-1], (N,)).to(cuda, torch.int32)
    idx = torch.randperm(N)[:n_items].to(cuda, torch.int32)
    p = _flat(_ref_net(dims)).to(cuda)
    P = mlp_num_params(dims)
    k = FusedMLPKernel(dims, bmax=4)
    nb = math.ceil(n_items / B)
    order = list(range(nb)) + [1, 2, 0]  # contiguous run, then a jump back
    stage = torch.zeros(256, dtype=torch.int32, device=cuda)
    cur_s = torch.zeros(1, dtype=torch.int32, device=cuda)
    cur_r = torch.zeros(1, dtype=torch.int32, device=cuda)
    for b in order:
        gs, gr = torch.zeros(P + 1, device=cuda), torch.zeros(P + 1, device=cuda)
        if int(cur_s.item()) != b:
            cur_s.fill_(b)
        cur_r.fill_(b)
        k.train(p, None, None, X, Y, idx, n_items=n_items, batch=B, steps=1, t0=0, lr=0.01, grad_out=gs,
                cursor=cur_s, stage=stage)
        k.train(p, None, None, X, Y, idx, n_items=n_items, batch=B, steps=1, t0=0, lr=0.01, grad_out=gr,
                cursor=cur_r)
        torch.cuda.synchronize()
        assert torch.equal(gs, gr), (b, (gs - gr).abs().max())
        assert int(cur_s.item()) == b + 1
        tag = int(stage[0].item())
        assert tag == (b + 2 if (b + 1) * B < n_items else 0), (b, tag)


@pytest.mark.parametrize("dropout,loss", [(0.0, "ce"), (0.2, "ce"), (0.2, "mse")])
def test_block5_two_micro_batch_kernel_equals_one_at_batch4(dropout, loss, cuda, monkeypatch):
    """mlp_block5's batch 5..8 kernels (two micro-batches of four rows per step, gradients summed in
    registers) forced at batch <= 4 (DCT_MLP_BLOCK=8): the second micro-batch's rows are all empty
    (zero dlogits), so every parameter, moment and loss must equal the one-micro-batch kernel's bit for
    bit - the partial last batch included (n_items % 4 = 3)."""
    torch.manual_seed(9)
    dims, N, n_items, B = [5, 128, 128, 2], 400, 203, 4
    X = torch.randn(N, 5).to(cuda)
    Y = torch.randint(0, 2, (N,)).to(cuda, torch.int32)
    idx = torch.randperm(N)[:n_items].to(cuda, torch.int32)
    p0 = _flat(_ref_net(dims)).to(cuda)
    steps = math.ceil(n_items / B)
    out = {}
    for blk in ("-1", "8"):
        monkeypatch.setenv("DCT_MLP_BLOCK", blk)
        p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
        losses = torch.zeros(steps, device=cuda)
        k = FusedMLPKernel(dims, bmax=4)
        for first, n in ((0, 17), (17, steps - 17)):  # two launches: the epilogue / prologue round trip too
            k.train(p, m, v, X, Y, idx[first * B:], n_items=n_items - first * B, batch=B, steps=n, t0=first, lr=0.01,
                    dropout=dropout, seed=3, step_base=first, loss=loss, loss_out=losses[first:])
        torch.cuda.synchronize()
        out[blk] = (p.cpu(), m.cpu(), v.cpu(), losses.cpu())
    for a_, b_ in zip(out["-1"], out["8"]):
        assert torch.isfinite(a_).all()
        assert torch.equal(a_, b_), float((a_ - b_).abs().max())


@pytest.mark.parametrize("dims,B,D0", [([7, 128, 128, 2], 4, 7), ([30, 128, 128, 3], 3, 30), ([5, 128, 128, 2], 8, 5),
                                      ([6, 128, 128, 2], 5, 6)])
def test_block_kernel_matches_lds_kernel_with_dropout(dims, B, D0, cuda, monkeypatch):
    """The register-resident 3-layer kernels (mlp_block5 where the shape fits, mlp_block3 with and
    without the 4x4x1 MFMA layer) vs the generic LDS kernel: same dropout hash, loss and Adam -> the
    same trajectory up to fp32 summation order."""
    torch.manual_seed(4)
    N, n_items = 500, 203
    X = torch.randn(N, D0).to(cuda)
    Y = torch.randint(0, dims[-1], (N,)).to(cuda, torch.int32)
    idx = torch.randperm(N)[:n_items].to(cuda, torch.int32)
    p0 = _flat(_ref_net(dims)).to(cuda)
    steps = math.ceil(n_items / B)
    out = {}
    variants = ("lds", "lds-b3", "lds-noblock")
    for blk in variants:
        _set_kernel_env(monkeypatch, blk)
        p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
        losses = torch.zeros(steps, device=cuda)
        k = FusedMLPKernel(dims, bmax=4 if B <= 4 else 16)
        k.train(p, m, v, X, Y, idx, n_items=n_items, batch=B, steps=steps, t0=3, lr=0.01, dropout=0.2, seed=11,
                step_base=5, loss_out=losses)
        torch.cuda.synchronize()
        out[blk] = (p.cpu(), m.cpu(), v.cpu(), losses.cpu())
    for blk in variants[:-1]:
        for a_, b_ in zip(out[blk], out["lds-noblock"]):
            assert torch.isfinite(a_).all()
            assert (a_ - b_).abs().max() <= 1e-4 * (1 + b_.abs().max()), (blk, float((a_ - b_).abs().max()))


@pytest.mark.parametrize("kernel", ["auto", "lds"])
def test_fused_dropout_keep_rate(kernel, cuda, monkeypatch):
    monkeypatch.setenv("DCT_MLP_KERNEL", kernel)
    # With dropout p the expected hidden activation is preserved (inverted scaling) and the
    # per-step masks differ; compare mean loss-gradient magnitude across many steps vs p=0.
    torch.manual_seed(3)
    dims = [8, 128, 2]
    N = 4096
    X = torch.randn(N, 8).abs()
    Y = torch.randint(0, 2, (N,))
    net = _ref_net(dims)
    with torch.no_grad():
        net[0].bias.fill_(1.0)
        net[0].weight.abs_()
    P = mlp_num_params(dims)
    k = FusedMLPKernel(dims, bmax=4)
    outs = []
    for pdrop in (0.0, 0.5):
        p = _flat(net).to(cuda)
        gsum = torch.zeros(P + 1, device=cuda)
        nz = 0
        for s in range(200):
            g = torch.zeros(P + 1, device=cuda)
            idx = torch.arange(s, s + 1, dtype=torch.int32, device=cuda)
            # batch of ONE row: a W2 gradient entry is zero exactly when its hidden unit was dropped
            k.train(p, None, None, X.to(cuda), Y.to(cuda, torch.int32), idx, n_items=1, batch=1, steps=1, t0=0,
                    lr=0.0, dropout=pdrop, seed=7, step_base=s, grad_out=g)
            w2 = g[8 * 128 + 128: 8 * 128 + 128 + 2 * 128].view(2, 128)
            nz += (w2.abs() > 0).float().mean().item()
            gsum += g
        outs.append(nz / 200)
    keep0, keep5 = outs
    assert keep0 > 0.99
    assert 0.40 < keep5 / keep0 < 0.60


def test_fused_eval_matches_torch(cuda):
    torch.manual_seed(4)
    dims = [5, 128, 128, 2]
    net = _ref_net(dims)
    N = 1000
    X = torch.randn(N, 5)
    Y = torch.randint(0, 2, (N,))
    idx = torch.randperm(N)[:777].to(torch.int32)
    k = FusedMLPKernel(dims, bmax=4)
    acc = torch.zeros(2, device=cuda)
    logits = torch.zeros(777 * 2, device=cuda)
    p = _flat(net).to(cuda)
    k.evaluate(p, X.to(cuda), Y.to(cuda, torch.int32), idx.to(cuda), 777, acc, logits_out=logits)
    z = net(X[idx.long()])
    assert torch.allclose(logits.view(777, 2).cpu(), z, atol=1e-4, rtol=1e-4)
    ls = F.cross_entropy(z, Y[idx.long()], reduction="sum").item()
    corr = (z.argmax(1) == Y[idx.long()]).sum().item()
    assert abs(acc[0].item() - ls) < 1e-2
    assert acc[1].item() == corr
    ref = reference_mlp_forward(p.cpu(), dims, X[:3])
    assert torch.allclose(ref, net(X[:3]), atol=1e-5)


def test_adam_flat_matches_torch(cuda):
    from dct_amd.ops.optim import adam_flat_

    torch.manual_seed(5)
    n = 1037
    w = torch.randn(n)
    net_p = torch.nn.Parameter(w.clone())
    opt = torch.optim.Adam([net_p], lr=0.01, weight_decay=0.1)
    p = w.clone().to(cuda)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    counter = torch.zeros(1, dtype=torch.int32, device=cuda)
    for t in range(1, 6):
        g = torch.randn(n)
        net_p.grad = g.clone()
        opt.step()
        if t % 2:
            adam_flat_(p, g.to(cuda), m, v, t, 0.01, weight_decay=0.1)
        else:  # device-counter path
            counter.fill_(t)
            adam_flat_(p, g.to(cuda), m, v, 1, 0.01, weight_decay=0.1, step_counter=counter)
    assert torch.allclose(p.cpu(), net_p.detach(), atol=1e-6, rtol=1e-5)


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 200, 72), (1, 17, 8), (257, 1024, 256), (64, 3, 1024),
                                   (136, 264, 128), (512, 256, 2048), (1024, 1024, 4096), (2, 1024, 512)])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_bf16(M, N, K, ta, tb, cuda):
    """fp32 out; covers the LDS-DMA/transpose-read fast path (K % 64 == 0), its split-K form
    (few tiles, long K) and the generic fallback (odd K / unaligned shapes)."""
    torch.manual_seed(6)
    A = torch.randn(M, K, device=cuda)
    B = torch.randn(K, N, device=cuda)
    As = A.t().contiguous() if ta else A.contiguous()
    Bs = B.t().contiguous() if tb else B.contiguous()
    As, Bs = _bf(As), _bf(Bs)
    C = torch.zeros(M, N, device=cuda)
    nat = native()
    nat.gemm_bf16(As.data_ptr(), Bs.data_ptr(), C.data_ptr(), 0, M, N, K, As.stride(0), Bs.stride(0), N, ta, tb, 0, 1,
                  0, 0, torch.cuda.current_stream().cuda_stream)
    ref = (As.float().t() if ta else As.float()) @ (Bs.float().t() if tb else Bs.float())
    torch.cuda.synchronize()
    assert torch.allclose(C, ref, atol=2e-3 * math.sqrt(K), rtol=1e-3)
    # accumulate=1 adds onto C (split-K slices add atomically onto the existing values)
    nat.gemm_bf16(As.data_ptr(), Bs.data_ptr(), C.data_ptr(), 0, M, N, K, As.stride(0), Bs.stride(0), N, ta, tb, 0, 1,
                  1, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.allclose(C, 2 * ref, atol=4e-3 * math.sqrt(K), rtol=2e-3)


@pytest.mark.parametrize("M,N,K,ta,tb,out_f32", [
    (2048, 1024, 1024, 0, 1, 0),  # 128 tiles x 16 k-tiles
    (1024, 768, 640, 0, 0, 0),    # NN (transposed-read B image), 10 k-tiles
    (512, 256, 8192, 1, 0, 1),    # dW shape: split-K slices of 8 k-tiles
    (768, 384, 192, 1, 0, 1),     # 3 k-tiles: prologue as deep as the whole loop
    (256, 512, 128, 0, 1, 0),     # 2 k-tiles: fewer tiles than pipeline stages
])
def test_gemm_pipeline_shapes(M, N, K, ta, tb, out_f32, cuda):
    """The two-stage LDS-DMA pipeline (counted vmcnt across a raw barrier) over loops longer and
    shorter than the pipeline, against the fp32 torch reference of the same bf16 operands."""
    torch.manual_seed(12)
    A = _bf(torch.randn(K, M, device=cuda) if ta else torch.randn(M, K, device=cuda))
    B = _bf(torch.randn(N, K, device=cuda) if tb else torch.randn(K, N, device=cuda))
    C = torch.empty(M, N, device=cuda, dtype=torch.float32 if out_f32 else torch.bfloat16)
    native().gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), 0, M, N, K, A.stride(0), B.stride(0), N, ta, tb, 0,
                       out_f32, 0, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = (A.float().t() if ta else A.float()) @ (B.float().t() if tb else B.float())
    tol = 2e-3 * math.sqrt(K) if out_f32 else 0.02 * math.sqrt(K)
    assert (C.float() - ref).abs().max().item() < tol, (C.float() - ref).abs().max().item()


@pytest.mark.parametrize("M,N,K,ta,tb", [
    (4096, 1024, 1024, 0, 1),  # tabular forward layer: 256 tiles, one per CU
    (4096, 1024, 1024, 0, 0),  # tabular dX layer (transposed-read B image)
    (4096, 1024, 256, 0, 1),   # tabular input layer: two 128-deep k stages
    (1024, 512, 256, 1, 0),    # transposed A image, 4 k-tiles (the prologue fills the whole loop)
    (2048, 2048, 512, 1, 1),   # transposed A image, KC B image, 256 tiles x 4 128-deep k stages
    (3000, 1024, 1024, 0, 1),  # 192 tiles, ragged M edge
    (300, 200, 512, 0, 1),     # ragged tile edges
])
def test_gemm_8wave_tiles(M, N, K, ta, tb, cuda):
    """One-tile-per-CU grids: 128 x 128 tiles worked by 8 waves (4 x 2, two per SIMD) with 2 LDS stages
    of 128-deep k (K >= 256) or the half-height two-per-CU tiles, with the bias + ReLU epilogue, bf16
    out, against the fp32 torch reference of the same bf16 operands."""
    torch.manual_seed(13)
    A = _bf(torch.randn(K, M, device=cuda) if ta else torch.randn(M, K, device=cuda))
    B = _bf(torch.randn(N, K, device=cuda) if tb else torch.randn(K, N, device=cuda))
    bias = torch.randn(N, device=cuda)
    C = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    native().gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), bias.data_ptr(), M, N, K, A.stride(0), B.stride(0), N,
                       ta, tb, 2, 0, 0, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = torch.relu((A.float().t() if ta else A.float()) @ (B.float().t() if tb else B.float()) + bias)
    assert (C.float() - ref).abs().max().item() < 0.02 * math.sqrt(K)


@pytest.mark.parametrize("M,N,K,accumulate,colsum", [
    (1024, 1024, 4096, 1, 1),  # tabular dW_l1: 64 tiles x 4 slices
    (1024, 256, 4096, 1, 1),   # tabular dW_l0: 16 tiles x 16 slices
    (192, 64, 32768, 0, 0),    # transformer dW (ungrouped): 2 tiles x 64 slices
    (200, 72, 2048, 1, 0),     # ragged tile edges, N % 4 == 0
    (136, 40, 1024, 0, 1),     # N % 8 == 0 only
])
def test_gemm_split_k_two_pass_and_atomic(M, N, K, accumulate, colsum, cuda):
    """Split-K dW (fp32 out, few tiles): two-pass for <= 4 slices per tile (slices store partials,
    one reduce kernel sums them in slice order), fp32 atomics above, against the fp32 torch
    reference, accumulating into an existing C and with the fused bias column sums."""
    torch.manual_seed(M + N)
    A = _bf(torch.randn(K, M, device=cuda))  # dZ [rows][M]
    B = _bf(torch.randn(K, N, device=cuda))  # X  [rows][N]
    C0 = torch.randn(M, N, device=cuda)
    C = C0.clone()
    cs0 = torch.randn(M, device=cuda)
    cs = cs0.clone()
    native().gemm_bf16_ex(A.data_ptr(), B.data_ptr(), C.data_ptr(), 0, M, N, K, M, N, N, 1, 0, 0, 1, accumulate, 0,
                          cs.data_ptr() if colsum else 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = A.float().t() @ B.float() + (C0 if accumulate else 0)
    tol = 2e-3 * math.sqrt(K)
    assert (C - ref).abs().max().item() < tol, (C - ref).abs().max().item()
    if colsum:
        assert torch.allclose(cs, cs0 + A.float().sum(0), atol=1e-2 * math.sqrt(K), rtol=1e-4)
    if (M, N) == (1024, 1024):  # two-pass (4 slices): fixed slice order, reproducible
        C2 = C0.clone()
        native().gemm_bf16_ex(A.data_ptr(), B.data_ptr(), C2.data_ptr(), 0, M, N, K, M, N, N, 1, 0, 0, 1, accumulate,
                              0, 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(C, C2)


@pytest.mark.parametrize("K", [640, 600])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0)])
def test_gemm_bf16_out_fast_and_generic_paths(ta, tb, K, cuda):
    """bf16 output of the LDS-DMA fast path (K a multiple of 64) and of the generic kernel (K = 600)
    against the fp32 torch reference."""
    torch.manual_seed(9)
    M, N = 384, 512
    A = _bf(torch.randn(K, M, device=cuda) if ta else torch.randn(M, K, device=cuda))
    B = _bf(torch.randn(N, K, device=cuda) if tb else torch.randn(K, N, device=cuda))
    C = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    native().gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), 0, M, N, K, A.stride(0), B.stride(0), N, ta, tb, 0, 0,
                       0, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = (A.float().t() if ta else A.float()) @ (B.float().t() if tb else B.float())
    assert torch.allclose(C.float(), ref, atol=0.3, rtol=2e-2)


@pytest.mark.parametrize("epi", [1, 2, 3])
def test_gemm_epilogues_and_accumulate(epi, cuda):
    torch.manual_seed(7)
    M, N, K = 200, 96, 128
    X = _bf(torch.randn(M, K, device=cuda))
    W = _bf(torch.randn(N, K, device=cuda) * 0.1)
    b = torch.randn(N, device=cuda)
    Y = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    aux = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    nat = native()
    nat.gemm_bf16(X.data_ptr(), W.data_ptr(), Y.data_ptr(), b.data_ptr(), M, N, K, K, K, N, 0, 1, epi, 0, 0,
                  aux.data_ptr(), torch.cuda.current_stream().cuda_stream)
    z = X.float() @ W.float().t() + b
    ref = {1: z, 2: torch.relu(z), 3: F.gelu(z)}[epi]
    torch.cuda.synchronize()
    assert torch.allclose(Y.float(), ref, atol=3e-2, rtol=2e-2)
    if epi == 3:
        assert torch.allclose(aux.float(), z, atol=3e-2, rtol=2e-2)
    # fp32 accumulate
    C = torch.ones(M, N, device=cuda)
    nat.gemm_bf16(X.data_ptr(), W.data_ptr(), C.data_ptr(), 0, M, N, K, K, K, N, 0, 1, 0, 1, 1, 0,
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.allclose(C, 1 + X.float() @ W.float().t(), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("act", [0, 1, 2])
def test_bias_act_bwd(act, cuda):
    torch.manual_seed(8)
    M, N = 333, 136
    dY = _bf(torch.randn(M, N, device=cuda))
    z = _bf(torch.randn(M, N, device=cuda))
    aux = z if act != 1 else _bf(torch.relu(z.float()))
    dZ = torch.empty_like(dY)
    db = torch.zeros(N, device=cuda)
    native().bias_act_bwd(dY.data_ptr(), aux.data_ptr(), dZ.data_ptr(), db.data_ptr(), M, N, N, act, 0,
                          torch.cuda.current_stream().cuda_stream)
    zz = z.float().requires_grad_(True)
    if act == 0:
        ref = dY.float()
    elif act == 1:
        ref = dY.float() * (aux.float() > 0)
    else:
        F.gelu(zz).backward(dY.float())
        ref = zz.grad
    torch.cuda.synchronize()
    assert torch.allclose(dZ.float(), ref, atol=2e-2, rtol=2e-2)
    assert torch.allclose(db, ref.sum(0), atol=0.3, rtol=2e-2)


@pytest.mark.parametrize("kind", [0, 1])
def test_loss_kernel(kind, cuda):
    torch.manual_seed(9)
    M, C = 1000, 3
    z = torch.randn(M, C, device=cuda)
    y = torch.randint(0, C, (M,), device=cuda)
    dz = torch.empty_like(z)
    ls = torch.zeros(1, device=cuda)
    cs = torch.zeros(1, device=cuda)
    native().cross_entropy_fwd_bwd(z.data_ptr(), 0, y.to(torch.int32).data_ptr(), dz.data_ptr(), ls.data_ptr(),
                                   cs.data_ptr(), M, C, 1.0 / M, kind, torch.cuda.current_stream().cuda_stream)
    zz = z.clone().requires_grad_(True)
    l = F.cross_entropy(zz, y) if kind == 0 else F.mse_loss(zz, F.one_hot(y, C).float())
    l.backward()
    torch.cuda.synchronize()
    assert abs(ls.item() / M - l.item()) < 1e-4
    assert torch.allclose(dz, zz.grad, atol=1e-6, rtol=1e-4)
    assert cs.item() == (z.argmax(1) == y).sum().item()


def test_layernorm_fwd_bwd(cuda):
    torch.manual_seed(10)
    M, N = 513, 192
    x = torch.randn(M, N, device=cuda)
    w = torch.randn(N, device=cuda)
    b = torch.randn(N, device=cuda)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=cuda)
    rstd = torch.empty(M, device=cuda)
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    nat.layernorm_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), M, N,
                      1e-5, 0, 0, st)
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    bb = b.clone().requires_grad_(True)
    ref = F.layer_norm(xx, (N,), ww, bb, 1e-5)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    dx = torch.empty_like(x)
    dw = torch.zeros(N, device=cuda)
    db = torch.zeros(N, device=cuda)
    nat.layernorm_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                      dw.data_ptr(), db.data_ptr(), M, N, 0, st)
    torch.cuda.synchronize()
    assert torch.allclose(y, ref.detach(), atol=1e-4, rtol=1e-4)
    assert torch.allclose(dx, xx.grad, atol=1e-4, rtol=1e-3)
    assert torch.allclose(dw, ww.grad, atol=1e-3, rtol=1e-3)
    assert torch.allclose(db, bb.grad, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("Bsz,H,T,D", [(2, 4, 6, 16), (3, 2, 33, 32), (1, 1, 256, 64), (5, 4, 64, 16), (3, 2, 32, 32),
                                       (2, 3, 48, 64), (7, 1, 16, 16), (2, 2, 80, 32)])
def test_attention_fwd_bwd(Bsz, H, T, D, cuda):
    """MFMA path (T, D multiples of 16, T <= 64) and the scalar LDS path (every other shape: T 6, 33,
    80, 256) against torch SDPA."""
    torch.manual_seed(11)
    dm = H * D
    qkv = _bf(torch.randn(Bsz * T, 3 * dm, device=cuda))
    o = torch.empty(Bsz * T, dm, device=cuda, dtype=torch.bfloat16)
    lse = torch.empty(Bsz * H * T, device=cuda)
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    scale = 1.0 / math.sqrt(D)
    q, k, v = (qkv[:, i * dm:(i + 1) * dm] for i in range(3))
    nat.attention_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), Bsz, H, T, D, 3 * dm,
                      dm, scale, st)

    def split(t):
        return t.float().reshape(Bsz, T, H, D).permute(0, 2, 1, 3)

    qq, kk, vv = (split(t).requires_grad_(True) for t in (q, k, v))
    ref = F.scaled_dot_product_attention(qq, kk, vv)
    torch.cuda.synchronize()
    got = o.float().reshape(Bsz, T, H, D).permute(0, 2, 1, 3)
    assert torch.allclose(got, ref.detach(), atol=2e-2, rtol=2e-2)
    do = _bf(torch.randn(Bsz * T, dm, device=cuda))
    ref.backward(split(do))
    dqkv = torch.zeros_like(qkv)
    dq, dk, dv = (dqkv[:, i * dm:(i + 1) * dm] for i in range(3))
    nat.attention_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                      dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), Bsz, H, T, D, 3 * dm, dm, scale, st)
    torch.cuda.synchronize()
    for g, r in ((dq, qq.grad), (dk, kk.grad), (dv, vv.grad)):
        gg = g.float().reshape(Bsz, T, H, D).permute(0, 2, 1, 3)
        assert torch.allclose(gg, r, atol=5e-2, rtol=5e-2), (gg - r).abs().max()


def test_gather_rows(cuda):
    src = torch.randn(1000, 12, device=cuda)
    idx = torch.randint(0, 1000, (333,), device=cuda, dtype=torch.int32)
    dst = torch.empty(333, 12, device=cuda)
    native().gather_rows(src.data_ptr(), idx.data_ptr(), dst.data_ptr(), 333, 48, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(dst, src[idx.long()])


def test_gemm_fused_bias_grad_and_mask_epilogues(cuda, monkeypatch):
    """dW GEMM with the bias gradient fused (colsum) and the dX GEMM's ReLU-mask / GELU' epilogues."""
    torch.manual_seed(10)
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    Bt, Dout, Din = 512, 256, 128
    for rows in (Bt, Bt - 12):  # the LDS-DMA path (rows % 64 == 0) and the generic kernel + column-sum kernel
        dZ = _bf(torch.randn(rows, Dout, device=cuda))
        A = _bf(torch.randn(rows, Din, device=cuda))
        dW = torch.zeros(Dout, Din, device=cuda)
        db = torch.zeros(Dout, device=cuda)
        nat.gemm_bf16_ex(dZ.data_ptr(), A.data_ptr(), dW.data_ptr(), 0, Dout, Din, rows, Dout, Din, Din, 1, 0, 0, 1,
                         1, 0, db.data_ptr(), st)
        torch.cuda.synchronize()
        assert torch.allclose(dW, dZ.float().t() @ A.float(), atol=0.1, rtol=1e-2)
        assert torch.allclose(db, dZ.float().sum(0), atol=0.05, rtol=1e-3)
    dZ = _bf(torch.randn(Bt, Dout, device=cuda))
    W = _bf(torch.randn(Dout, Din, device=cuda) * 0.1)
    act = _bf(torch.relu(torch.randn(Bt, Din, device=cuda)))
    out = torch.empty(Bt, Din, device=cuda, dtype=torch.bfloat16)
    nat.gemm_bf16(dZ.data_ptr(), W.data_ptr(), out.data_ptr(), 0, Bt, Din, Dout, Dout, Din, Din, 0, 0,
                  nat.EPI_RELU_MASK, 0, 0, act.data_ptr(), st)
    torch.cuda.synchronize()
    ref = (dZ.float() @ W.float()) * (act.float() > 0)
    assert torch.allclose(out.float(), ref, atol=5e-2, rtol=2e-2)
    pre = _bf(torch.randn(Bt, Din, device=cuda))
    nat.gemm_bf16(dZ.data_ptr(), W.data_ptr(), out.data_ptr(), 0, Bt, Din, Dout, Dout, Din, Din, 0, 0,
                  nat.EPI_GELU_GRAD, 0, 0, pre.data_ptr(), st)
    torch.cuda.synchronize()
    z = pre.float().requires_grad_(True)
    F.gelu(z).backward(dZ.float() @ W.float())
    assert torch.allclose(out.float(), z.grad, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("C", [1, 2, 3, 8])
def test_skinny_head_kernels(C, cuda):
    torch.manual_seed(11)
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    Bt, K = 777, 1024
    X = _bf(torch.randn(Bt, K, device=cuda))
    W = _bf(torch.randn(C, K, device=cuda) * 0.05)
    b = torch.randn(C, device=cuda)
    Y = torch.empty(Bt, C, device=cuda, dtype=torch.bfloat16)
    nat.skinny_fwd(X.data_ptr(), W.data_ptr(), b.data_ptr(), Y.data_ptr(), Bt, K, C, st)
    dZ = _bf(torch.randn(Bt, C, device=cuda))
    act = _bf(torch.relu(torch.randn(Bt, K, device=cuda)))
    dX = torch.empty(Bt, K, device=cuda, dtype=torch.bfloat16)
    nat.skinny_dx(dZ.data_ptr(), W.data_ptr(), act.data_ptr(), dX.data_ptr(), Bt, K, C, st)
    dW = torch.zeros(C, K, device=cuda)
    db = torch.zeros(C, device=cuda)
    nat.skinny_dw(dZ.data_ptr(), X.data_ptr(), dW.data_ptr(), db.data_ptr(), Bt, K, C, st)
    torch.cuda.synchronize()
    assert torch.allclose(Y.float(), X.float() @ W.float().t() + b, atol=3e-2, rtol=2e-2)
    assert torch.allclose(dX.float(), (dZ.float() @ W.float()) * (act.float() > 0), atol=2e-2, rtol=2e-2)
    assert torch.allclose(dW, dZ.float().t() @ X.float(), atol=5e-2, rtol=1e-3)
    assert torch.allclose(db, dZ.float().sum(0), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("B,K,C,kind", [(4096, 1024, 2, 0), (4096, 1024, 2, 1), (777, 1024, 2, 0), (333, 512, 1, 1),
                                        (100, 2048, 2, 0), (130, 1024, 3, 0), (65, 512, 8, 0), (4096, 1536, 2, 1)])
def test_fused_skinny_head_matches_fp32_reference_and_chain(B, K, C, kind, cuda):
    """csrc/skinny.hip skinny_head_kernel (head fwd + CE/MSE + dlogits + dW/db + masked dH in one
    launch) against (a) a plain torch fp32 reference of the same op and (b) the unfused chain
    skinny_fwd -> loss -> skinny_dw -> skinny_dx it replaces in the tabular step executor."""
    torch.manual_seed(B + K + C)
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    assert nat.skinny_head_supported(K, C)
    H = _bf(torch.relu(torch.randn(B, K, device=cuda)))
    W = _bf(torch.randn(C, K, device=cuda) * 0.03)
    b = torch.randn(C, device=cuda) * 0.1
    y = torch.randint(0, C, (B,), device=cuda).to(torch.int32)
    dH = torch.empty(B, K, device=cuda, dtype=torch.bfloat16)
    dW = torch.zeros(C, K, device=cuda)
    db = torch.zeros(C, device=cuda)
    ls = torch.zeros(1, device=cuda)
    nat.skinny_head(H.data_ptr(), W.data_ptr(), b.data_ptr(), y.data_ptr(), dH.data_ptr(), dW.data_ptr(),
                    db.data_ptr(), ls.data_ptr(), B, K, C, 1.0 / B, kind, 1.0 / B, 1, st)
    # (b) the unfused chain on the same operands
    Z = torch.empty(B, C, device=cuda, dtype=torch.bfloat16)
    nat.skinny_fwd(H.data_ptr(), W.data_ptr(), b.data_ptr(), Z.data_ptr(), B, K, C, st)
    dZ = torch.empty(B, C, device=cuda, dtype=torch.bfloat16)
    ls2 = torch.zeros(1, device=cuda)
    nat.cross_entropy_fwd_bwd(Z.data_ptr(), 1, y.data_ptr(), dZ.data_ptr(), ls2.data_ptr(), 0, B, C, 1.0 / B, kind, st)
    dW2 = torch.zeros(C, K, device=cuda)
    db2 = torch.zeros(C, device=cuda)
    nat.skinny_dw(dZ.data_ptr(), H.data_ptr(), dW2.data_ptr(), db2.data_ptr(), B, K, C, st)
    dH2 = torch.empty(B, K, device=cuda, dtype=torch.bfloat16)
    nat.skinny_dx(dZ.data_ptr(), W.data_ptr(), H.data_ptr(), dH2.data_ptr(), B, K, C, st)
    # (a) fp32 reference
    z = (H.float() @ W.float().t() + b).requires_grad_(True)
    loss = _ref_loss(z, y.long(), "ce" if kind == 0 else "mse")
    loss.backward()
    dz = z.grad
    torch.cuda.synchronize()
    assert abs(ls.item() - loss.item()) < 2e-3 * max(1.0, abs(loss.item()))
    assert abs(ls.item() - ls2.item() / B) < 1e-5 * max(1.0, abs(loss.item()))  # same bf16 logits, same math
    assert torch.allclose(dW, dz.t() @ H.float(), atol=2e-3, rtol=2e-2)
    assert torch.allclose(db, dz.sum(0), atol=2e-3, rtol=2e-2)
    ref_dH = (dz @ W.float()) * (H.float() > 0)
    assert torch.allclose(dH.float(), ref_dH, atol=1e-4, rtol=2e-2)
    # chain parity: bf16 logits / dlogits rounded identically, only atomic summation order differs
    assert torch.equal(dH, dH2)
    assert torch.allclose(dW, dW2, atol=1e-6, rtol=1e-5)
    assert torch.allclose(db, db2, atol=1e-6, rtol=1e-5)


def test_fused_head_executor_step_matches_unfused(cuda, monkeypatch):
    """The wide-MLP step executor with the fused head (default) and with DCT_FUSED_HEAD=0 (the
    four-kernel chain) train the same trajectory (eager steps and captured graphs alike)."""
    from dct_amd.models.mlp import MLPClassifier
    from dct_amd.parallel.dist import init_distributed
    from dct_amd.trainer.engines import adam_hparams_from
    from dct_amd.trainer.graph_engine import GraphMLPEngine

    ctx = init_distributed("gpu")
    dims, B = [256, 1024, 1024, 2], 512
    g = torch.Generator().manual_seed(0)
    X = torch.randn(12 * B, dims[0], generator=g)
    Y = ((X @ torch.randn(dims[0], generator=g)) > 0).long()
    rows = torch.arange(X.shape[0])
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("DCT_FUSED_HEAD", fused)
        torch.manual_seed(0)
        model = MLPClassifier(dims[0], hidden=tuple(dims[1:-1]), num_classes=2, dropout=0.0, loss="ce", lr=1e-3)
        eng = GraphMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
        eng.attach_data(X, Y, rows, rows[:B])
        losses = torch.cat([eng.train_epoch(ep).cpu() for ep in range(2)])
        torch.cuda.synchronize()
        res[fused] = (losses, eng.p.cpu())
    (l1, p1), (l0, p0) = res["1"], res["0"]
    assert torch.isfinite(l1).all() and l1[-4:].mean() < l1[:4].mean()
    assert torch.allclose(l1, l0, atol=1e-3), (l1 - l0).abs().max()
    assert (p1 - p0).norm() / p0.norm() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("M,d,n", [(4096, 64, 256), (1000, 64, 128)])
def test_ffn_residual_matches_fp32_reference(cuda, M, d, n):
    """ops.nn.ffn_residual (4 GEMMs, gelu' + bias grads in epilogues) vs an fp32 torch reference."""
    from dct_amd.ops.nn import ffn_residual

    torch.manual_seed(0)
    a = torch.randn(M, d, device=cuda).to(torch.bfloat16).requires_grad_()
    h = torch.randn(M, d, device=cuda, requires_grad=True)
    w1 = (torch.randn(n, d, device=cuda) / math.sqrt(d)).requires_grad_()
    b1 = (0.1 * torch.randn(n, device=cuda)).requires_grad_()
    w2 = (torch.randn(d, n, device=cuda) / math.sqrt(n)).requires_grad_()
    b2 = (0.1 * torch.randn(d, device=cuda)).requires_grad_()
    dout = torch.randn(M, d, device=cuda)
    out = ffn_residual(a, w1, b1, w2, b2, h)
    out.backward(dout)
    leaves = [a, w1, b1, w2, b2, h]
    got = [t.grad.float().clone() for t in leaves]
    for t in leaves:
        t.grad = None
    ref = h + F.linear(F.gelu(F.linear(a.float(), w1, b1)), w2, b2)
    ref.backward(dout)
    torch.cuda.synchronize()
    assert (out - ref).norm() / ref.norm() < 1e-2
    for name, g, t in zip(["a", "w1", "b1", "w2", "b2", "h"], got, leaves):
        rel = (g - t.grad.float()).norm() / (t.grad.float().norm() + 1e-12)
        assert rel < 2e-2, (name, float(rel))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(32768, 64), (1000, 128), (77, 256)])
def test_layernorm_bwd_fused_residual_and_slots(cuda, M, N):
    """layernorm_bwd_ex: bf16 dy, fp32 x, + dres, bf16 copy of dx, dw/db accumulated through the
    slot workspace (run twice: the kernel must leave the workspace zeroed for the next call)."""
    from dct_amd.ops.nn import _ln_ws

    torch.manual_seed(11)
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    x = torch.randn(M, N, device=cuda)
    w = torch.randn(N, device=cuda)
    b = torch.randn(N, device=cuda)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    dy16 = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    dres = torch.randn(M, N, device=cuda)
    xx, ww, bb = (t.clone().requires_grad_(True) for t in (x, w, b))
    F.layer_norm(xx, (N,), ww, bb, 1e-5).backward(dy16.float())
    ws = _ln_ws(x.device, N)
    dw = torch.full((N,), 0.5, device=cuda)  # accumulates (+=) into existing grads
    db = torch.zeros(N, device=cuda)
    for it in range(2):
        dx = torch.empty_like(x)
        dx16 = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        nat.layernorm_bwd_ex(dy16.data_ptr(), 1, x.data_ptr(), 0, w.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                             dx.data_ptr(), 0, dx16.data_ptr(), dres.data_ptr(), dw.data_ptr(), db.data_ptr(),
                             ws.data_ptr(), M, N, st)
        torch.cuda.synchronize()
        ref_dx = xx.grad + dres
        assert torch.allclose(dx, ref_dx, atol=1e-3, rtol=1e-3), it
        assert torch.equal(dx16, dx.to(torch.bfloat16))
        assert torch.allclose(dw, 0.5 + (it + 1) * ww.grad, atol=2e-2, rtol=1e-3), it
        assert torch.allclose(db, (it + 1) * bb.grad, atol=2e-2, rtol=1e-3), it
    assert int(ws.count_nonzero()) == 0


def _prenorm_inputs(cuda, M, d, n, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(cuda).requires_grad_()  # noqa: E731
    return dict(h=mk(M, d), ln_w=(1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_(), ln_b=mk(d, scale=0.1),
                w1=mk(n, d, scale=d ** -0.5), b1=mk(n, scale=0.1), w2=mk(d, n, scale=n ** -0.5), b2=mk(d, scale=0.1))


@pytest.mark.gpu
@pytest.mark.parametrize("bound", [False, True])
def test_prenorm_ffn_matches_fp32_reference(cuda, bound):
    """ops.nn.prenorm_ffn (one fused autograd node) vs fp32 torch; bound=True routes the
    parameter gradients through bound_params' direct accumulation into pre-set .grad buffers."""
    from dct_amd.ops.nn import bound_params, prenorm_ffn

    M, d, n = 4096, 64, 256
    t = _prenorm_inputs(cuda, M, d, n)
    params = [t[k] for k in ("ln_w", "ln_b", "w1", "b1", "w2", "b2")]
    dout = torch.randn(M, d, device=cuda)
    if bound:
        for p in params:
            p.grad = torch.zeros_like(p)
        with bound_params(params):
            out = prenorm_ffn(t["h"], *params)
            out.backward(dout)
    else:
        out = prenorm_ffn(t["h"], *params)
        out.backward(dout)
    got = {k: v.grad.clone() for k, v in t.items()}
    for v in t.values():
        v.grad = None
    a = F.layer_norm(t["h"], (d,), t["ln_w"], t["ln_b"], 1e-5)
    ref = t["h"] + F.linear(F.gelu(F.linear(a, t["w1"], t["b1"])), t["w2"], t["b2"])
    ref.backward(dout)
    torch.cuda.synchronize()
    assert (out - ref).norm() / ref.norm() < 1e-2
    for k, v in t.items():
        rel = (got[k] - v.grad).norm() / (v.grad.norm() + 1e-12)
        assert rel < 3e-2, (k, float(rel))


@pytest.mark.gpu
def test_prenorm_attention_matches_fp32_reference(cuda):
    from dct_amd.ops.nn import prenorm_attention

    B, T, H, d = 128, 32, 4, 64
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(3)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(cuda).requires_grad_()  # noqa: E731
    t = dict(h=mk(M, d), ln_w=(1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_(), ln_b=mk(d, scale=0.1),
             wqkv=mk(3 * d, d, scale=d ** -0.5), bqkv=mk(3 * d, scale=0.1), wo=mk(d, d, scale=d ** -0.5),
             bo=mk(d, scale=0.1))
    dout = torch.randn(M, d, device=cuda)
    out = prenorm_attention(t["h"], t["ln_w"], t["ln_b"], t["wqkv"], t["bqkv"], t["wo"], t["bo"], B, H, T)
    out.backward(dout)
    got = {k: v.grad.clone() for k, v in t.items()}
    for v in t.values():
        v.grad = None
    a = F.layer_norm(t["h"], (d,), t["ln_w"], t["ln_b"], 1e-5)
    q, k, v = (z.reshape(B, T, H, d // H).transpose(1, 2) for z in F.linear(a, t["wqkv"], t["bqkv"]).split(d, 1))
    o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(M, d)
    ref = t["h"] + F.linear(o, t["wo"], t["bo"])
    ref.backward(dout)
    torch.cuda.synchronize()
    assert (out - ref).norm() / ref.norm() < 1e-2
    for name, tv in t.items():
        rel = (got[name] - tv.grad).norm() / (tv.grad.norm() + 1e-12)
        assert rel < 4e-2, (name, float(rel))


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 37, 512])
def test_tt_block_fused_matches_fp32_reference_and_unfused(cuda, B, monkeypatch):
    """ops.nn.tt_block at the TabTransformer shape (64 tokens, d 64, 4 heads, FFN 256): the
    whole-block kernels (csrc/tt_block.hip: forward, and the backward dX chain + split-K dW GEMMs)
    vs an fp32 torch block, and vs the unfused two-node path - outputs and every gradient."""
    from dct_amd.ops import nn as nnops

    T, H, d, n = 64, 4, 64, 256
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(11)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(cuda).requires_grad_()  # noqa: E731
    t = dict(h=mk(M, d), ln1_w=(1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_(),
             ln1_b=mk(d, scale=0.1), wqkv=mk(3 * d, d, scale=d ** -0.5), bqkv=mk(3 * d, scale=0.1),
             wo=mk(d, d, scale=d ** -0.5), bo=mk(d, scale=0.1),
             ln2_w=(1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_(), ln2_b=mk(d, scale=0.1),
             w1=mk(n, d, scale=d ** -0.5), b1=mk(n, scale=0.1), w2=mk(d, n, scale=n ** -0.5), b2=mk(d, scale=0.1))
    keys = ["ln1_w", "ln1_b", "wqkv", "bqkv", "wo", "bo", "ln2_w", "ln2_b", "w1", "b1", "w2", "b2"]
    dout = torch.randn(M, d, device=cuda)

    def run(fused, fused_bwd=True):
        monkeypatch.setattr(nnops, "TT_FUSED", fused)
        monkeypatch.setattr(nnops, "TT_FUSED_BWD", fused_bwd)
        assert nnops.tt_block_fusable(t["h"], H, T, n) == fused
        out = nnops.tt_block(t["h"], *[t[k] for k in keys], B, H, T)
        out.backward(dout)
        grads = {k: v.grad.clone() for k, v in t.items()}
        for v in t.values():
            v.grad = None
        return out.detach(), grads

    monkeypatch.setattr(nnops, "TT_FUSED", True)
    with torch.no_grad():  # inference mode of the block kernel: only the output is written
        out_inf = nnops.tt_block(t["h"], *[t[k] for k in keys], B, H, T)
    out_f, g_f = run(True)               # fused forward + fused backward kernel
    assert torch.equal(out_inf, out_f)
    out_fu, g_fu = run(True, False)      # fused forward + the unfused backward nodes
    out_u, g_u = run(False)
    a = F.layer_norm(t["h"], (d,), t["ln1_w"], t["ln1_b"], 1e-5)
    q, k, v = (z.reshape(B, T, H, d // H).transpose(1, 2) for z in F.linear(a, t["wqkv"], t["bqkv"]).split(d, 1))
    o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(M, d)
    h1 = t["h"] + F.linear(o, t["wo"], t["bo"])
    a2 = F.layer_norm(h1, (d,), t["ln2_w"], t["ln2_b"], 1e-5)
    ref = h1 + F.linear(F.gelu(F.linear(a2, t["w1"], t["b1"])), t["w2"], t["b2"])
    ref.backward(dout)
    torch.cuda.synchronize()
    assert torch.isfinite(out_f).all()
    assert (out_f - ref).norm() / ref.norm() < 1e-2
    assert (out_f - out_u).norm() / out_u.norm() < 2e-3  # same bf16 roundings, different sum order
    for name, tv in t.items():
        rel = (g_f[name] - tv.grad).norm() / (tv.grad.norm() + 1e-12)
        assert rel < 5e-2, (name, float(rel))
        rel_u = (g_f[name] - g_u[name]).norm() / (g_u[name].norm() + 1e-12)
        assert rel_u < 2e-2, (name, float(rel_u))
        rel_fu = (g_fu[name] - g_u[name]).norm() / (g_u[name].norm() + 1e-12)
        assert rel_fu < 2e-2, (name, float(rel_fu))


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("B,C", [(1, 2), (37, 2), (512, 2), (64, 5)])
def test_tt_embed_and_head_loss_match_fp32_reference(cuda, B, C, fused):
    """csrc/tt_io.hip: feature-token embedding fwd/bwd and the pooled LN -> Linear -> mean-CE head
    (loss forward, recomputing backward) vs fp32 torch, every gradient including dh.  ``fused``: the
    training forward under unit_loss_seed() (backward seed 1) - loss and gradients from ONE launch
    (dct_tt_head_fused), the backward only hands them over."""
    import contextlib

    from dct_amd.ops.nn import tt_embed, tt_head_loss, unit_loss_seed

    F_, d = 64, 64
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(B, F_, generator=g).to(cuda)
    y = torch.randint(0, C, (B,), generator=g).to(cuda)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(cuda).requires_grad_()  # noqa: E731
    E, c = mk(F_, d, scale=0.2), mk(F_, d, scale=0.1)
    lw = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    lb, W, bias = mk(d, scale=0.1), mk(C, d, scale=0.3), mk(C, scale=0.1)
    params = [E, c, lw, lb, W, bias]
    with unit_loss_seed() if fused else contextlib.nullcontext():
        h = tt_embed(x, E, c)
        h2 = h * 1.5  # an op between embedding and head, so dh flows through autograd
        loss = tt_head_loss(h2, y, B, F_, lw, lb, W, bias, root=True)
        loss.backward(torch.ones_like(loss))
    got = [p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    hr = (x[:, :, None] * E + c).reshape(B * F_, d) * 1.5
    z = F.layer_norm(hr.reshape(B, F_, d).mean(1), (d,), lw, lb, 1e-5)
    ref = F.cross_entropy(F.linear(z, W, bias), y)
    ref.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 1e-4 * max(1.0, abs(ref.item()))
    for p, gg in zip(params, got):
        rel = (gg - p.grad).norm() / (p.grad.norm() + 1e-12)
        assert rel < 1e-3, float(rel)


@pytest.mark.gpu
def test_tt_head_loss_repeated_launches_deterministic(cuda):
    """tt_io.hip head_fwd_kernel: the last workgroup (ticket count) sums the per-workgroup partials in
    block order and stores the loss, leaving the ticket at zero - so back-to-back launches of any batch
    size (the scratch grows past its first size) give the fp32 reference loss, bit-identical on
    repeats, without a zero-filled loss tensor."""
    from dct_amd.ops.nn import tt_head_loss, unit_loss_seed

    F_, d, C = 64, 64, 2
    g = torch.Generator(device="cpu").manual_seed(11)
    lw = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda)
    lb, W, bias = (0.1 * torch.randn(d, generator=g)).to(cuda), (0.3 * torch.randn(C, d, generator=g)).to(cuda), \
        (0.1 * torch.randn(C, generator=g)).to(cuda)
    for B in (512, 3, 1100, 512, 64):
        h = torch.randn(B * F_, d, generator=g).to(cuda)
        y = torch.randint(0, C, (B,), generator=g).to(cuda)
        with torch.no_grad():
            losses = [tt_head_loss(h, y, B, F_, lw, lb, W, bias) for _ in range(3)]
            z = F.layer_norm(h.reshape(B, F_, d).mean(1), (d,), lw, lb, 1e-5)
            ref = F.cross_entropy(F.linear(z, W, bias), y)
        torch.cuda.synchronize()
        vals = [float(t) for t in losses]
        assert vals[0] == vals[1] == vals[2], (B, vals)
        assert abs(vals[0] - ref.item()) < 1e-4 * max(1.0, abs(ref.item())), (B, vals[0], ref.item())
        # the fused training forward (loss + gradients in one launch) stores the same loss, bit for bit
        hg = h.clone().requires_grad_()
        with unit_loss_seed():
            lf = tt_head_loss(hg, y, B, F_, lw.requires_grad_(), lb.requires_grad_(), W.requires_grad_(),
                              bias.requires_grad_(), root=True)
        assert float(lf) == vals[0], (B, float(lf), vals[0])
        lw.requires_grad_(False), lb.requires_grad_(False), W.requires_grad_(False), bias.requires_grad_(False)


@pytest.mark.gpu
@pytest.mark.parametrize("accumulate", [0, 1])
@pytest.mark.parametrize("grouped", [True, False])
def test_gemm_dw_grouped(cuda, accumulate, grouped):
    """dct_gemm_bf16_dw_grouped: four dW = dZ^T X products (+ bias column sums) of different shapes
    in one split-K launch (4096 rows), and the per-problem fallback it takes when a problem has too
    few k-tiles to split (256 rows), vs fp32 torch."""
    from dct_amd.ops._native import native

    g = torch.Generator(device="cpu").manual_seed(9)
    rows = 4096 if grouped else 256
    shapes = [(64, 256), (256, 64), (64, 64), (192, 64)]
    dz = [torch.randn(rows, m, generator=g).to(cuda).to(torch.bfloat16) for m, _ in shapes]
    xs = [torch.randn(rows, n, generator=g).to(cuda).to(torch.bfloat16) for _, n in shapes]
    c0 = [torch.randn(m, n, generator=g).to(cuda) for m, n in shapes]
    cs0 = [torch.randn(m, generator=g).to(cuda) for m, _ in shapes]
    C = [c.clone() if accumulate else torch.full_like(c, 7.0) for c in c0]
    CS = [c.clone() for c in cs0]
    st = torch.cuda.current_stream().cuda_stream
    native().gemm_bf16_dw_grouped([t.data_ptr() for t in dz], [t.data_ptr() for t in xs], [t.data_ptr() for t in C],
                                  [m for m, _ in shapes], [n for _, n in shapes], rows, [t.data_ptr() for t in CS],
                                  accumulate, st)
    torch.cuda.synchronize()
    for i in range(4):
        ref = dz[i].float().t() @ xs[i].float() + (c0[i] if accumulate else 0)
        assert (C[i] - ref).norm() / ref.norm() < 1e-3, i
        assert torch.allclose(CS[i], cs0[i] + dz[i].float().sum(0), rtol=1e-3, atol=1e-2), i


@pytest.mark.gpu
def test_skinny_head_linear_and_shadow_weights(cuda):
    """ops.nn.linear with N <= 8 takes the skinny kernels; under bound_params a registered bf16
    shadow replaces the weight conversion and gradients accumulate into .grad."""
    from dct_amd.ops.nn import bound_params, linear

    torch.manual_seed(5)
    x = torch.randn(512, 64, device=cuda).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(2, 64, device=cuda) / 8).requires_grad_()
    b = torch.randn(2, device=cuda).requires_grad_()
    dy = torch.randn(512, 2, device=cuda)
    w.grad, b.grad = torch.ones_like(w), torch.zeros_like(b)
    shadow = torch.zeros(2, 64, dtype=torch.bfloat16, device=cuda)
    shadow.copy_(w.detach())
    with bound_params([w, b], {id(w): shadow}):
        y = linear(x, w, b)
        y.float().backward(dy)
    ref = F.linear(x.float(), w, b)
    gx = x.grad.clone()
    gw, gb = w.grad.clone(), b.grad.clone()
    x.grad = w.grad = b.grad = None
    ref.backward(dy)
    torch.cuda.synchronize()
    assert torch.allclose(y.float(), ref, atol=3e-2, rtol=2e-2)
    # dy is rounded to bf16 for the kernels: compare by relative norm, not elementwise
    assert (gw - 1.0 - w.grad).norm() / w.grad.norm() < 1e-2
    assert (gb - b.grad).norm() / b.grad.norm() < 1e-2
    assert (gx.float() - x.grad.float()).norm() / x.grad.float().norm() < 1e-2


@pytest.mark.parametrize("dims", [[5, 64, 2], [5, 128, 128, 2]])
def test_bound_train_launch_matches_keyword_launch(dims, cuda):
    """BoundTrain (operands bound once, run(first_step, steps)) trains exactly like the keyword
    launch over the same slices of the index list, including the loss slots and step counter."""
    torch.manual_seed(1)
    P = mlp_num_params(dims)
    k = FusedMLPKernel(dims, bmax=4)
    N = 512
    X = torch.randn(N, dims[0], device=cuda)
    Y = torch.randint(0, dims[-1], (N,), device=cuda, dtype=torch.int32)
    idx = torch.randperm(N, device=cuda).to(torch.int32)
    p0 = torch.randn(P, device=cuda) * 0.2
    runs = []
    for bound in (False, True):
        p, m, v = p0.clone(), torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
        ctr = torch.zeros(1, dtype=torch.int32, device=cuda)
        loss = torch.full((64,), -1.0, device=cuda)
        if bound:
            bl = k.prepare_train(p, m, v, X, Y, idx, n_items=N, batch=4, lr=0.01, dropout=0.2, seed=7,
                                 loss_out=loss, step_counter=ctr)
            bl.run(0, 5)
            bl.run(5, 20)
            with pytest.raises(Exception):
                bl.run(60, 10)  # past the loss buffer
        else:
            for first, steps in ((0, 5), (5, 20)):
                k.train(p, m, v, X, Y, idx[first * 4:], n_items=N - first * 4, batch=4, steps=steps, t0=0, lr=0.01,
                        dropout=0.2, seed=7, loss_out=loss[first:first + steps], step_counter=ctr)
        torch.cuda.synchronize()
        runs.append((p, m, v, loss, ctr))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    assert int(runs[1][4]) == 25 and bool((runs[1][3][:25] > 0).all()) and bool((runs[1][3][25:] == -1).all())


@pytest.mark.gpu
@pytest.mark.parametrize("B", [512, 1024])
def test_tt_ln_replica_fold_complete_and_matches_direct_atomics(cuda, B, monkeypatch):
    """ADVICE r5 (csrc/tt_block.hip LN_REP fold): the fused block backward adds each workgroup's
    LayerNorm parameter gradients into one of 16 replicas and the LAST workgroup (ticket) folds them
    with memory-side read-and-zero atomics, ordered only by ``s_waitcnt vmcnt(0)`` behind the adds (no
    release fence: an agent-scope release writes back the XCD's L2, 0.339 -> 0.556 ms per step).  A
    replica add that landed after the fold would stay in the workspace: after every launch the
    replicas and the ticket must be exactly zero, and the folded gradients must equal the direct-
    atomic path's up to fp32 summation order (a lost workgroup would move a column by ~1/sqrt(B) of it)."""
    from dct_amd.ops import nn as nnops

    T, H, d, n = 64, 4, 64, 256
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(3)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(cuda).requires_grad_()  # noqa: E731
    t = dict(h=mk(M, d), ln1_w=(1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_(),
             ln1_b=mk(d, scale=0.1), wqkv=mk(3 * d, d, scale=d ** -0.5), bqkv=mk(3 * d, scale=0.1),
             wo=mk(d, d, scale=d ** -0.5), bo=mk(d, scale=0.1),
             ln2_w=(1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_(), ln2_b=mk(d, scale=0.1),
             w1=mk(n, d, scale=d ** -0.5), b1=mk(n, scale=0.1), w2=mk(d, n, scale=n ** -0.5), b2=mk(d, scale=0.1))
    keys = ["ln1_w", "ln1_b", "wqkv", "bqkv", "wo", "bo", "ln2_w", "ln2_b", "w1", "b1", "w2", "b2"]
    ln_keys = ["ln1_w", "ln1_b", "ln2_w", "ln2_b"]
    dout = torch.randn(M, d, device=cuda)
    monkeypatch.setattr(nnops, "TT_FUSED", True)
    monkeypatch.setattr(nnops, "TT_FUSED_BWD", True)

    def run(rep):
        monkeypatch.setattr(nnops, "_TT_LN_REP", rep)
        out = nnops.tt_block(t["h"], *[t[k] for k in keys], B, H, T)
        out.backward(dout)
        grads = {k: t[k].grad.clone() for k in ln_keys}
        for v in t.values():
            v.grad = None
        return grads

    direct = run(False)
    for it in range(8):
        got = run(True)
        torch.cuda.synchronize()
        ws = nnops._TT_LN_WS[cuda.index if cuda.index is not None else 0]
        assert int(torch.count_nonzero(ws)) == 0, (it, int(torch.count_nonzero(ws)))  # replicas + ticket re-zeroed
        for k in ln_keys:
            err = (got[k] - direct[k]).abs().max()
            assert err <= 2e-4 * direct[k].abs().max() + 1e-6, (it, k, float(err), float(direct[k].abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("M", [4096, 300])
def test_gemm_forward_wt_side_output_and_nt_dx(cuda, M):
    """The wide MLP's forward GEMM side output (csrc/gemm_bf16.hip dct_gemm_bf16_bt): W^T written from
    the LDS B images (bt_out) equals W.t() bit for bit, and the dX GEMM the executor runs on it - NT on
    W^T - equals the NN form on W (both with the bf16-activation ReLU mask, EPI_RELU_MASK) bit for bit."""
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(5)
    N, K = 1024, 512
    X = (torch.randn(M, K, device=cuda) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=cuda) * 0.1
    Y = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    WT = torch.zeros(K, N, device=cuda, dtype=torch.bfloat16)
    nat.gemm_bf16_bt(X.data_ptr(), W.data_ptr(), Y.data_ptr(), b.data_ptr(), M, N, K, K, K, N, nat.EPI_BIAS_RELU, 0,
                     0, WT.data_ptr(), N, st)
    torch.cuda.synchronize()
    assert torch.equal(WT, W.t().contiguous())
    ref = torch.relu(X.float() @ W.float().t() + b)
    assert (Y.float() - ref).abs().max() < 2e-2 * ref.abs().max()
    # dX of the NEXT layer: dZ [M][N2] (W2 [N2][N]) -> dX [M][N] masked by relu'(Y)
    N2 = 1024
    dZ = (torch.randn(M, N2, device=cuda) * 0.1).to(torch.bfloat16)
    W2 = (torch.randn(N2, N, device=cuda) * 0.05).to(torch.bfloat16)
    W2T = W2.t().contiguous()
    d_nn = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    d_nt = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    nat.gemm_bf16(dZ.data_ptr(), W2.data_ptr(), d_nn.data_ptr(), 0, M, N, N2, N2, N, N, 0, 0, nat.EPI_RELU_MASK, 0, 0,
                  Y.data_ptr(), st)
    nat.gemm_bf16(dZ.data_ptr(), W2T.data_ptr(), d_nt.data_ptr(), 0, M, N, N2, N2, N2, N, 0, 1, nat.EPI_RELU_MASK, 0, 0,
                  Y.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(d_nn, d_nt)
    want = (dZ.float() @ W2.float()) * (Y.float() > 0)
    assert (d_nt.float() - want).abs().max() < 2e-2 * want.abs().max()


@pytest.mark.gpu
def test_tt_head_loss_not_root_keeps_the_backward_launch(cuda):
    """Under unit_loss_seed() only a head loss declared the backward root (root=True) computes its
    gradients in the forward launch: a caller that scales the loss before backward (root left False)
    gets the scaled gradients from the backward launch."""
    from dct_amd.ops.nn import tt_head_loss, unit_loss_seed

    B, T_, d, C = 96, 1, 64, 2
    g = torch.Generator(device="cpu").manual_seed(21)
    h0 = torch.randn(B * T_, d, generator=g).to(cuda)
    y = torch.randint(0, C, (B,), generator=g).to(cuda)
    lw = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda)
    lb, W, bias = (0.1 * torch.randn(d, generator=g)).to(cuda), (0.3 * torch.randn(C, d, generator=g)).to(cuda), \
        (0.1 * torch.randn(C, generator=g)).to(cuda)
    grads = []
    for scale, ctxm in ((1.0, False), (0.5, True)):
        h = h0.clone().requires_grad_()
        Wp = W.clone().requires_grad_()
        with unit_loss_seed() if ctxm else torch.enable_grad():
            loss = tt_head_loss(h, y, B, T_, lw, lb, Wp, bias) * scale
            loss.backward(torch.ones_like(loss))
        torch.cuda.synchronize()
        grads.append((h.grad.clone(), Wp.grad.clone()))
    (dh1, dW1), (dh5, dW5) = grads
    assert torch.allclose(dh5, 0.5 * dh1, rtol=1e-5, atol=1e-8)
    assert torch.allclose(dW5, 0.5 * dW1, rtol=1e-5, atol=1e-7)
