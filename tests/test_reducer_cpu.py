"""Reducer assumptions that hold on any device, pinned on CPU:

* the fused ops accumulate weight gradients straight into ``p.grad`` and return ``None`` to
  autograd (ops/nn.py bound_params); torch still runs the post-accumulate-grad hooks for such
  parameters, so the bucket reducer's hooks (trainer/engines.py AutogradEngine) fire during
  backward and launch buckets before ``finalize`` (the overlap the GPU test measures);
* bucket planning: reverse parameter order, first bucket capped at first_bucket_bytes.
"""
import torch

from dct_amd.parallel.reducer import TorchBucketReducer, plan_buckets


class _DirectGrad(torch.autograd.Function):
    """y = x @ w with dW accumulated in place into w.grad and None returned for it."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        w.grad.add_(x.t() @ g)
        return g @ w.t(), None


def test_post_accumulate_hooks_fire_for_in_place_grads():
    torch.manual_seed(0)
    ws = [torch.nn.Parameter(torch.randn(8, 8)) for _ in range(3)]
    flat = torch.zeros(3 * 64)
    for i, w in enumerate(ws):
        w.grad = flat[i * 64:(i + 1) * 64].view(8, 8)
    plan = plan_buckets([64, 64, 64], 4, bucket_cap_bytes=256, first_bucket_bytes=256)
    assert plan.counts == [64, 64, 64] and plan.param_bucket == [2, 1, 0]
    red = TorchBucketReducer(flat, plan, world_size=1)
    order = []

    def hook(i):
        def h(_p):
            order.append((i, red.mark_ready(i)))
        return h

    for i, w in enumerate(ws):
        w.register_post_accumulate_grad_hook(hook(i))
    x = torch.randn(4, 8)
    h = x
    for w in ws:
        h = torch.relu(_DirectGrad.apply(h, w))
    h.sum().backward()
    # every hook fired, last layer first, and each completed its bucket during backward
    assert [i for i, _ in order] == [2, 1, 0]
    assert all(n == 1 for _, n in order)
    assert red.next == red.num_buckets  # nothing left for finalize to launch
    red.finalize()
    ref = [torch.nn.Parameter(w.detach().clone()) for w in ws]
    h = x
    for w in ref:
        h = torch.relu(h @ w)
    h.sum().backward()
    for w, r in zip(ws, ref):
        assert torch.allclose(w.grad, r.grad, atol=1e-5)


def test_plan_buckets_split_before_aligns_buckets_with_groups():
    """split_before closes the bucket being filled (reverse parameter order) before a parameter:
    the TabTransformer's block groups become their own buckets regardless of the byte caps."""
    plan = plan_buckets([10, 20, 30, 40, 50], 4, bucket_cap_bytes=1 << 20, first_bucket_bytes=1 << 20,
                        split_before=[2])
    assert plan.param_bucket == [1, 1, 1, 0, 0]
    assert plan.offsets == [60, 0] and plan.counts == [90, 60]
    # without the split: one bucket
    assert plan_buckets([10, 20, 30, 40, 50], 4, 1 << 20, 1 << 20).param_bucket == [0] * 5


def test_tabtransformer_block_groups_split_the_ddp_buckets(monkeypatch):
    """AutogradEngine._block_groups on the TabTransformer (DCT_TT_DDP_GROUPS=1; off by default): the
    upper half of the blocks (with the head) and the lower half (with the embedding) as two bucket
    groups; the split index is the last parameter of the highest block of the lower group."""
    from dct_amd.models.tabtransformer import TabTransformer
    from dct_amd.parallel.dist import DistContext
    from dct_amd.trainer.engines import AutogradEngine

    m = TabTransformer(num_features=8, d_model=16, heads=2, layers=4)
    assert m.ddp_block_groups() == [[3, 2], [1, 0]]
    assert TabTransformer(num_features=8, d_model=16, heads=2, layers=3).ddp_block_groups() == [[2, 1], [0]]
    assert TabTransformer(num_features=8, d_model=16, heads=2, layers=1).ddp_block_groups() is None
    params = list(m.parameters())

    class _Eng:
        ctx = DistContext(rank=0, world_size=2)

    monkeypatch.delenv("DCT_TT_DDP_GROUPS", raising=False)
    assert AutogradEngine._block_groups(_Eng(), m, params) == ((), ())  # default: one group
    monkeypatch.setenv("DCT_TT_DDP_GROUPS", "1")
    groups, splits = AutogradEngine._block_groups(_Eng(), m, params)
    assert groups == (2, 2)
    first_b2 = [i for i, p in enumerate(params) if p is next(m.blocks[2].parameters())][0]
    assert splits == (first_b2 - 1,)
    plan = plan_buckets([p.numel() for p in params], 4, 8 << 20, 1 << 20, split_before=splits)
    assert len(plan.counts) == 2
    upper = {id(p) for b in (2, 3) for p in m.blocks[b].parameters()} | {id(p) for p in m.head.parameters()}
    for i, p in enumerate(params):
        assert plan.param_bucket[i] == (0 if id(p) in upper or i > first_b2 else 1)


def test_block_group_buckets_never_split_inside_a_group(monkeypatch):
    """A TabTransformer whose per-block weights exceed the first-bucket / bucket caps (d_model 192:
    one block's 12 d^2 fp32 weights are ~1.7 MB > 1 MiB) must still get exactly one bucket per
    block group: the group's dW GEMMs are issued only inside its lowest block's backward, so a
    bucket covering part of a group would be all-reduced before its gradients are written."""
    from dct_amd.models.tabtransformer import TabTransformer
    from dct_amd.parallel.dist import DistContext
    from dct_amd.trainer.engines import AutogradEngine

    monkeypatch.setenv("DCT_TT_DDP_GROUPS", "1")
    for d, layers in ((192, 4), (64, 12)):
        m = TabTransformer(num_features=8, d_model=d, heads=4, layers=layers)
        params = list(m.parameters())

        class _Eng:
            ctx = DistContext(rank=0, world_size=2)

        groups, splits = AutogradEngine._block_groups(_Eng(), m, params)
        plan = plan_buckets([p.numel() for p in params], 4, 1 << 20, 256 << 10, split_before=splits)
        assert len(plan.counts) == len(groups) == 2
        group_of = {}
        for g, blocks in enumerate(m.ddp_block_groups()):
            for b in blocks:
                for p in m.blocks[b].parameters():
                    group_of[id(p)] = g
        for i, p in enumerate(params):
            if id(p) in group_of:
                assert plan.param_bucket[i] == group_of[id(p)], (d, layers, i)
        # every bucket is a contiguous slice and together they cover the flat buffer once
        assert sum(plan.counts) == sum(p.numel() for p in params)


def test_executor_buckets_close_at_layer_boundaries():
    """The wide-MLP executor's DDP buckets (trainer/graph_engine.py layer_bucket_splits): whole
    layers from the top until >= 2 MiB, so the last bucket - the only all-reduce that cannot overlap
    backward - is the input layer alone."""
    from dct_amd.trainer.graph_engine import layer_bucket_splits

    dims = [256, 1024, 1024, 1024, 2]
    numels = []
    for i in range(len(dims) - 1):
        numels += [dims[i] * dims[i + 1], dims[i + 1]]
    splits = layer_bucket_splits(numels, 8 << 20)
    plan = plan_buckets(numels + [1], 4, 8 << 20, 1 << 20, split_before=splits)
    # params: W0 b0 W1 b1 W2 b2 W3 b3 loss -> buckets {W2 b2 W3 b3 loss}, {W1 b1}, {W0 b0}
    assert plan.param_bucket == [2, 2, 1, 1, 0, 0, 0, 0, 0]
    assert plan.counts[-1] == 256 * 1024 + 1024
