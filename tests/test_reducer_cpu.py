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
