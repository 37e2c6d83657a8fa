"""Flat-buffer Adam (reference: ``torch.optim.Adam(self.parameters(), lr=0.01)``,
jobs/train_lightning_ddp.py:87-88).

Every parameter of the model is a view into ONE flat fp32 buffer (and every ``.grad`` a view
into one flat gradient buffer, which is what the bucketed reducer all-reduces), so a step
is one fused kernel launch on the GPU (csrc/optim.hip) or one vectorised torch expression on
the CPU plumbing path.  ``state_dict()`` emits exactly torch.optim.Adam's format so the
Lightning checkpoint's ``optimizer_states`` entry stays loadable by torch 2.1 / Lightning 2.1.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from ._native import native, ptr, stream_handle


def adam_flat_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
               betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, grad_scale: float = 1.0,
               decoupled: bool = False, p_bf16: Optional[torch.Tensor] = None,
               step_counter: Optional[torch.Tensor] = None):
    """In-place Adam on flat fp32 buffers; ``step`` is the 1-based step count after this update."""
    n = p.numel()
    for t in (g, m, v):
        if t.numel() != n or t.dtype != torch.float32 or not t.is_contiguous() or t.device != p.device:
            raise ValueError("adam_flat_: p/g/m/v must be contiguous fp32 buffers of equal size on one device")
    if p.is_cuda:
        if p_bf16 is not None and (p_bf16.dtype != torch.bfloat16 or p_bf16.numel() != n):
            raise ValueError("p_bf16 must be a bf16 buffer of the same size")
        if step_counter is not None and not (step_counter.is_cuda and step_counter.dtype == torch.int32):
            raise ValueError("step_counter must be a cuda int32 tensor")
        native().adam_flat(ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), n, float(lr), float(betas[0]),
                           float(betas[1]), float(eps), float(weight_decay), max(1, int(step)), float(grad_scale),
                           int(decoupled), ptr(step_counter), stream_handle(p.device))
        return
    b1, b2 = betas
    gg = g * grad_scale if grad_scale != 1.0 else g
    if decoupled:
        p.mul_(1 - lr * weight_decay)
    elif weight_decay:
        gg = gg + weight_decay * p
    m.mul_(b1).add_(gg, alpha=1 - b1)
    v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if p_bf16 is not None:
        p_bf16.copy_(p)


def _torch_adam_group_defaults() -> Dict:
    """The param-group keys the installed ``torch.optim.Adam`` writes (they vary by torch
    version, e.g. ``decoupled_weight_decay`` since 2.6), so our optimizer state dicts stay
    loadable by ``torch.optim.Adam.load_state_dict`` and by Lightning."""
    try:
        d = dict(torch.optim.Adam([torch.zeros(1, requires_grad=True)]).defaults)
    except Exception:  # noqa: BLE001
        d = dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, maximize=False,
                 foreach=None, capturable=False, differentiable=False, fused=None)
    return d


class FlatAdam:
    """Adam over a flat parameter buffer, torch.optim.Adam-compatible state_dict."""

    def __init__(self, flat_param: torch.Tensor, flat_grad: torch.Tensor, param_shapes: Sequence[torch.Size],
                 lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported")
        self.p = flat_param
        self.g = flat_grad
        self.m = torch.zeros_like(flat_param)
        self.v = torch.zeros_like(flat_param)
        self.shapes = [torch.Size(s) for s in param_shapes]
        group = _torch_adam_group_defaults()
        group.update(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                     params=list(range(len(self.shapes))))
        self.param_groups = [group]
        self.step_count = 0
        self.p_bf16: Optional[torch.Tensor] = None

    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    def step(self, grad_scale: float = 1.0, bump_counter: bool = True, epilogue=None):
        """One update.  ``bump_counter=False``: a step-prologue kernel already advanced the device
        step counter.  ``epilogue=(cursor, loss, loss_out)``: the Adam kernel also records
        loss_out[*cursor] = loss and advances the device batch cursor (graph-replayed loops)."""
        self.step_count += 1
        g = self.param_groups[0]
        counter = None
        if self.p.is_cuda:
            # the Adam step count lives on the device (advanced by a kernel, read by the Adam
            # kernel), so a captured step graph replays with the right bias correction
            counter = self._device_counter()
            if bump_counter:
                counter.add_(1)
        if epilogue is not None:
            cursor, loss, loss_out = epilogue
            b1, b2 = g["betas"]
            native().adam_flat_step(ptr(self.p), ptr(self.g), ptr(self.m), ptr(self.v), ptr(self.p_bf16),
                                    self.p.numel(), float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                    float(g["weight_decay"]), max(1, self.step_count), float(grad_scale), 0,
                                    ptr(counter), ptr(cursor), ptr(loss), ptr(loss_out), loss_out.numel(),
                                    stream_handle(self.p.device))
            return
        adam_flat_(self.p, self.g, self.m, self.v, self.step_count, g["lr"], g["betas"], g["eps"],
                   g["weight_decay"], grad_scale=grad_scale, p_bf16=self.p_bf16, step_counter=counter)

    def _device_counter(self) -> torch.Tensor:
        c = getattr(self, "_counter", None)
        if c is None or c.device != self.p.device:
            self._counter = c = torch.full((1,), self.step_count - 1, dtype=torch.int32, device=self.p.device)
        return c

    def sync_device_counter(self):
        """Re-seed the device step counter from the host count (after a state load)."""
        if self.p.is_cuda:
            self._device_counter().fill_(self.step_count)

    def zero_grad(self):
        self.g.zero_()

    # ------------------------------------------------------------------ state dict
    def _views(self, flat):
        out, off = [], 0
        for s in self.shapes:
            n = s.numel()
            out.append(flat[off: off + n].view(s))
            off += n
        return out

    def state_dict(self) -> Dict:
        state = {}
        if self.step_count > 0:
            ms, vs = self._views(self.m), self._views(self.v)
            for i in range(len(self.shapes)):
                state[i] = {
                    "step": torch.tensor(float(self.step_count)),
                    "exp_avg": ms[i].detach().to("cpu", torch.float32).clone(),
                    "exp_avg_sq": vs[i].detach().to("cpu", torch.float32).clone(),
                }
        groups = []
        for g in self.param_groups:
            gg = dict(g)
            gg["betas"] = tuple(gg["betas"])
            groups.append(gg)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd: Dict):
        pg = sd["param_groups"][0]
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in pg:
                self.param_groups[0][k] = tuple(pg[k]) if k == "betas" else pg[k]
        st = sd.get("state", {})
        if st:
            ms, vs = self._views(self.m), self._views(self.v)
            steps = set()
            for i in range(len(self.shapes)):
                s = st[i] if i in st else st[str(i)]
                ms[i].copy_(s["exp_avg"])
                vs[i].copy_(s["exp_avg_sq"])
                steps.add(int(float(s["step"])))
            self.step_count = max(steps)
        else:
            self.step_count = 0
        if getattr(self, "_counter", None) is not None:
            self._counter.fill_(self.step_count)
