"""Autograd functions over the native HIP kernels (bf16 activations, fp32 master weights).

Used by the transformer-style models (models/tabtransformer.py) on MI355X:
  * ``linear``     - MFMA GEMM forward with fused bias / ReLU / GELU epilogue; backward = two
                     GEMMs (dX = dZ W, dW = dZ^T X with the bias gradient fused as a column sum)
                     and one elementwise activation-derivative pass when needed;
  * ``ffn_residual`` - the GELU MLP sub-block with gelu' and both bias gradients fused into GEMMs;
  * ``prenorm_attention`` / ``prenorm_ffn`` - whole pre-norm residual sub-blocks as single
                     autograd nodes (LayerNorm backward fused with the residual-gradient add);
  * ``layer_norm`` - one wave per row, fp32 statistics (fwd) / fused dX, dgamma, dbeta (bwd);
  * ``attention``  - fused feature-token attention over a packed QKV projection (online softmax
                     forward, recompute backward).
On CPU (the gloo plumbing config) the same functions fall back to plain torch ops; on a GPU the
native module is required (``native()`` raises if it is missing - no silent fallback).
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Dict, Iterable, List, Optional, Sequence

import torch
import torch.nn.functional as F

from ._native import native

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2
_EPI = {ACT_NONE: 1, ACT_RELU: 2, ACT_GELU: 3}  # EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_GELU
EPI_GELU_GRAD = 5
_SKINNY_MAX = 8  # csrc/skinny.hip SK_CMAX


def _stream():
    return torch.cuda.current_stream().cuda_stream


# ----------------------------------------------------------------------------- engine binding
class _Binding:
    def __init__(self, params: Iterable[torch.Tensor], shadows: Optional[Dict[int, torch.Tensor]],
                 defer_dw: bool = False, defer_groups: Sequence[int] = ()):
        self.direct = {id(p) for p in params}
        self.shadows = shadows or {}
        self.defer_dw = defer_dw
        # deferred dW flush points: block counts (backward order) after which the queued dW GEMMs
        # are issued right away, e.g. (2, 2) for 4 blocks - see bound_params
        self.flush_at = set()
        acc = 0
        for n in defer_groups:
            acc += int(n)
            self.flush_at.add(acc)
        self.deferred_blocks = 0


_BOUND: Optional[_Binding] = None


@contextlib.contextmanager
def bound_params(params: Iterable[torch.Tensor], bf16_shadows: Optional[Dict[int, torch.Tensor]] = None,
                 defer_dw: bool = False, defer_groups: Sequence[int] = ()):
    """Engine-scoped fast paths for the ops below (trainer/engines.py AutogradEngine):

    * gradient accumulation fusion - the weight-gradient GEMMs / LayerNorm column sums of a
      bound parameter ACCUMULATE straight into ``p.grad`` (a view of the flat DDP bucket
      buffer, zeroed once per step) and the op returns ``None`` for it, so there is no per-
      parameter gradient tensor, fill or AccumulateGrad add.  Post-accumulate-grad hooks still
      fire (autograd runs them for undefined gradients too), so bucket all-reduces launch as before;
    * bf16 shadow weights - ``bf16_shadows[id(p)]`` (kept current by the fused Adam) replaces
      the per-step fp32->bf16 weight conversion;
    * ``defer_dw`` - the fused transformer block's weight-gradient GEMMs are queued and issued by
      :func:`join_side_work` as ONE grouped split-K launch for every block after backward.  (Running
      them on a side stream under the earlier blocks' backward measured slower, 0.420 -> 0.445 ms,
      profiles/tabular_dw_side_stream_ab_r2.log / tt_head_spb_side_dw_ab_r2.log; removed.);
    * ``defer_groups`` (with ``defer_dw``) - block counts in backward order after which the queued
      GEMMs are issued at once, INSIDE the backward of the block closing the group: with a DDP
      bucket reducer whose buckets follow the same groups (plan_buckets ``split_before``), the
      group's bucket is complete - and launches from its hooks - when that block's backward
      returns, so its all-reduce overlaps the earlier blocks' backward.
    """
    global _BOUND
    # leftovers of a backward that never reached join_side_work (an aborted graph capture) belong
    # to that step: issuing them into this step's gradients would corrupt it
    _SIDE["deferred"].clear()
    _SIDE.pop("embed", None)
    prev, _BOUND = _BOUND, _Binding(params, bf16_shadows, defer_dw, defer_groups)
    try:
        yield
    finally:
        _BOUND = prev


# deferred weight-gradient work (bound_params(defer_dw=True)): the queued dW GEMMs with the operand
# tensors they read (kept referenced until they are issued)
_SIDE = {"deferred": []}


def join_side_work():
    """Issue the deferred dW GEMMs (bound_params(defer_dw=True)) as grouped launches of up to 16."""
    _flush_deferred()


def _flush_deferred():
    """Issue the queued dW GEMMs as grouped launches of up to 16 problems (stream order), with a
    queued embedding-gradient job (the fused first block's) riding in the first."""
    dfr = _SIDE["deferred"]
    emb = _SIDE.pop("embed", None)
    if not dfr and emb is None:
        return
    nat, st = native(), _stream()
    if dfr:
        for i in range(0, len(dfr), 16):
            _dw_gemm_grouped(nat, dfr[i:i + 16], st, embed=emb if i == 0 else None)
        dfr.clear()
    elif emb is not None:
        _embed_bwd(nat, emb, st)


def _w16(w: torch.Tensor) -> torch.Tensor:
    b = _BOUND
    if b is not None:
        sh = b.shadows.get(id(w))
        if sh is not None and sh.data_ptr() % 16 == 0:  # the MFMA / skinny paths stage 16-B rows
            return sh
    return w.detach().to(torch.bfloat16).contiguous()


def _is_direct(p: torch.Tensor) -> bool:
    """True when p's gradient accumulates straight into the bound p.grad (see bound_params)."""
    b = _BOUND
    if b is None or id(p) not in b.direct:
        return False
    g = p.grad
    return g is not None and g.dtype == torch.float32 and g.is_contiguous() and g.shape == p.shape


def _grad_dst(p: torch.Tensor, zero: bool = False):
    """(buffer, direct): p.grad itself when accumulation into it is bound, else a new tensor."""
    if _is_direct(p):
        return p.grad, True
    alloc = torch.zeros if zero else torch.empty
    return alloc(p.shape, dtype=torch.float32, device=p.device), False


# the bf16 copy of the last residual-stream gradient a fused LayerNorm backward produced: the
# next (earlier) block's backward receives exactly that fp32 tensor as its output gradient
_BF16_PAIR = None


def _remember_bf16(t32: torch.Tensor, t16: torch.Tensor):
    global _BF16_PAIR
    _BF16_PAIR = (t32, t32._version, t16)


def _bf16_of(t: torch.Tensor) -> torch.Tensor:
    pr = _BF16_PAIR
    if pr is not None:
        t32, ver, t16 = pr
        if t32 is t or (t32.data_ptr() == t.data_ptr() and t32.shape == t.shape and t32.stride() == t.stride()
                        and t.dtype == torch.float32 and t._version == ver):
            return t16
    t = t.contiguous()
    return t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16)


_LN_WS: Dict[tuple, torch.Tensor] = {}


def _ln_ws(device: torch.device, N: int) -> torch.Tensor:
    """Persistent zeroed slot workspace of the fused LayerNorm backward (re-zeroed by the kernel)."""
    key = (device.index, N)
    ws = _LN_WS.get(key)
    if ws is None:
        ws = torch.zeros(native().layernorm_bwd_ws_floats(N), dtype=torch.float32, device=device)
        _LN_WS[key] = ws
    return ws


def _ln_fused_ok(N: int) -> bool:
    return N % 4 == 0 and N <= 256


def _ln_bwd(nat, dy16, x, w, b, mean, rstd, dres=None, want_bf16=False):
    """Fused narrow LayerNorm backward: dx fp32 (+ dres) [+ bf16 copy]; dw/db into w/b grads."""
    M, N = x.shape
    dx = torch.empty(M, N, dtype=torch.float32, device=x.device)
    dx16 = torch.empty(M, N, dtype=torch.bfloat16, device=x.device) if want_bf16 else None
    dw, dw_direct = _grad_dst(w, zero=True)
    db, db_direct = _grad_dst(b, zero=True)
    nat.layernorm_bwd_ex(dy16.data_ptr(), 1, x.data_ptr(), 0, w.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                         dx.data_ptr(), 0, dx16.data_ptr() if dx16 is not None else 0,
                         dres.data_ptr() if dres is not None else 0, dw.data_ptr(), db.data_ptr(),
                         _ln_ws(x.device, N).data_ptr(), M, N, _stream())
    if dx16 is not None:
        _remember_bf16(dx, dx16)
    return dx, None if dw_direct else dw, None if db_direct else db


def _dw_gemm(nat, dz16, x16, w, b, st):
    """dW (+)= dZ^T X with the bias gradient (+)= colsum(dZ) fused; returns the non-direct grads."""
    M, N = dz16.shape
    K = x16.shape[1]
    dw, dw_direct = _grad_dst(w)
    db, db_direct = _grad_dst(b, zero=True)
    nat.gemm_bf16_ex(dz16.data_ptr(), x16.data_ptr(), dw.data_ptr(), 0, N, K, M, N, K, K, 1, 0, 0, 1,
                     1 if dw_direct else 0, 0, db.data_ptr(), st)
    return None if dw_direct else dw, None if db_direct else db


def _embed_bwd(nat, emb, st):
    x, dh, dE, dc, B, F, dm = emb
    nat.tt_embed_bwd(x.data_ptr(), dh.data_ptr(), dE.data_ptr(), dc.data_ptr(), B, F, dm, st)


def _dw_gemm_grouped(nat, items, st, embed=None):
    """Several dW (+)= dZ^T X products over the same rows (bias grads fused) in ONE launch
    (csrc/gemm_bf16.hip dct_gemm_bf16_dw_grouped); returns [(dw, db)] with None for direct grads."""
    rows = items[0][0].shape[0]
    dws, dbs, out = [], [], []
    for dz16, x16, w, b in items:
        assert dz16.shape[0] == rows and x16.shape[0] == rows
        dw, dw_direct = _grad_dst(w, zero=True)  # zeroed when not direct: the launch accumulates
        db, db_direct = _grad_dst(b, zero=True)
        dws.append(dw)
        dbs.append(db)
        out.append((None if dw_direct else dw, None if db_direct else db))
    args = ([it[0].data_ptr() for it in items], [it[1].data_ptr() for it in items], [d.data_ptr() for d in dws],
            [it[0].shape[1] for it in items], [it[1].shape[1] for it in items], rows, [d.data_ptr() for d in dbs], 1)
    if embed is None:
        nat.gemm_bf16_dw_grouped(*args, st)
    else:  # the embedding gradients ride in the launch (csrc/gemm_bf16.hip EmbedRide), else on their own
        x, dh, dE, dc, B, F, dm = embed
        if not nat.gemm_bf16_dw_grouped_embed(*args, x.data_ptr(), dh.data_ptr(), dE.data_ptr(), dc.data_ptr(),
                                              B, F, st):
            _embed_bwd(nat, embed, st)
    return out


def _mm(nat, a16, b16, M, N, K, st, epi=0, aux=None, out=None):
    """C[M, N] = A[M, K] B[K, N] (bf16 out) with an optional elementwise backward epilogue."""
    c = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=a16.device)
    nat.gemm_bf16(a16.data_ptr(), b16.data_ptr(), c.data_ptr(), 0, M, N, K, K, N, N, 0, 0, epi, 0, 0,
                  aux.data_ptr() if aux is not None else 0, st)
    return c


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act):
        nat = native()
        x = x.contiguous()
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        M, K = x.shape
        N = weight.shape[0]
        wb = _w16(weight)
        st = _stream()
        y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        ctx.skinny = act == ACT_NONE and N <= _SKINNY_MAX and K % 8 == 0
        pre = None
        if ctx.skinny:  # classifier heads: a bandwidth kernel, not a 128x128 MFMA tile
            nat.skinny_fwd(x.data_ptr(), wb.data_ptr(), bias.data_ptr(), y.data_ptr(), M, K, N, st)
        else:
            pre = torch.empty_like(y) if act == ACT_GELU else None
            nat.gemm_bf16(x.data_ptr(), wb.data_ptr(), y.data_ptr(), bias.data_ptr(), M, N, K, K, K, N, 0, 1,
                          _EPI[act], 0, 0, pre.data_ptr() if pre is not None else 0, st)
        ctx.act = act
        ctx.save_for_backward(x, wb, y if act == ACT_RELU else pre)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        nat = native()
        x, wb, aux = ctx.saved_tensors
        weight, bias = ctx.params
        act = ctx.act
        dy = _bf16_of(dy)
        M, K = x.shape
        N = wb.shape[0]
        st = _stream()
        dx = None
        if ctx.skinny:
            dw, dw_direct = _grad_dst(weight, zero=True)
            db, db_direct = _grad_dst(bias, zero=True)
            nat.skinny_dw(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(), M, K, N, st)
            if ctx.needs_input_grad[0]:
                dx = torch.empty(M, K, dtype=torch.bfloat16, device=x.device)
                nat.skinny_dx(dy.data_ptr(), wb.data_ptr(), 0, dx.data_ptr(), M, K, N, st)
            return dx, None if dw_direct else dw, None if db_direct else db, None
        if act == ACT_NONE:
            dz = dy
            dw, db = _dw_gemm(nat, dz, x, weight, bias, st)
        else:  # dZ = dY * act'(.) and db in one pass
            dz = torch.empty_like(dy)
            db, db_direct = _grad_dst(bias, zero=True)
            nat.bias_act_bwd(dy.data_ptr(), aux.data_ptr(), dz.data_ptr(), db.data_ptr(), M, N, N, act, 1, st)
            dw, dw_direct = _grad_dst(weight)
            nat.gemm_bf16_ex(dz.data_ptr(), x.data_ptr(), dw.data_ptr(), 0, N, K, M, N, K, K, 1, 0, 0, 1,
                             1 if dw_direct else 0, 0, 0, st)
            dw = None if dw_direct else dw
            db = None if db_direct else db
        if ctx.needs_input_grad[0]:
            dx = _mm(nat, dz, wb, M, K, N, st)
        return dx, dw, db, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, act: int = ACT_NONE) -> torch.Tensor:
    """y = act(x W^T + b); x [M, K] (bf16 on GPU), W [N, K] fp32, b [N] fp32."""
    if x.is_cuda:
        return _LinearFn.apply(x, weight, bias, act)
    y = F.linear(x.float(), weight, bias)
    return F.relu(y) if act == ACT_RELU else (F.gelu(y) if act == ACT_GELU else y)


class _LinearResidualFn(torch.autograd.Function):
    """out = h + x W^T + b in fp32 from one GEMM epilogue (the residual-stream update)."""

    @staticmethod
    def forward(ctx, x, weight, bias, h):
        nat = native()
        x = x.contiguous()
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        h = h.contiguous().float()
        M, K = x.shape
        N = weight.shape[0]
        wb = _w16(weight)
        out = torch.empty(M, N, dtype=torch.float32, device=x.device)
        nat.gemm_bf16_residual(x.data_ptr(), wb.data_ptr(), out.data_ptr(), bias.data_ptr(), h.data_ptr(), M, N, K,
                               _stream())
        ctx.save_for_backward(x, wb)
        ctx.params = (weight, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        nat = native()
        x, wb = ctx.saved_tensors
        weight, bias = ctx.params
        M, K = x.shape
        N = wb.shape[0]
        st = _stream()
        dz = _bf16_of(dout)
        dw, db = _dw_gemm(nat, dz, x, weight, bias, st)
        dx = _mm(nat, dz, wb, M, K, N, st) if ctx.needs_input_grad[0] else None
        return dx, dw, db, dout


def linear_residual(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """h + x W^T + b (fp32): on GPU one GEMM with the residual folded into its epilogue."""
    if x.is_cuda:
        return _LinearResidualFn.apply(x, weight, bias, h)
    return h.float() + F.linear(x.float(), weight, bias)


def _ffn_fwd(nat, a, w1b, b1, w2b, b2, h, st):
    M, K = a.shape
    N = w1b.shape[0]
    f = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    pre = torch.empty_like(f)
    nat.gemm_bf16(a.data_ptr(), w1b.data_ptr(), f.data_ptr(), b1.data_ptr(), M, N, K, K, K, N, 0, 1, _EPI[ACT_GELU],
                  0, 0, pre.data_ptr(), st)
    out = torch.empty(M, K, dtype=torch.float32, device=a.device)
    nat.gemm_bf16_residual(f.data_ptr(), w2b.data_ptr(), out.data_ptr(), b2.data_ptr(), h.data_ptr(), M, K, N, st)
    return f, pre, out


def _ffn_bwd(nat, dz2, a, w1b, w2b, f, pre, params, st, want_da=True):
    """Backward of h + W2 gelu(W1 a + b1) + b2 from dZ2 (bf16): gelu' in the dF GEMM epilogue,
    both bias gradients as dW-GEMM column sums -> (da, dw1, db1, dw2, db2)."""
    w1, b1, w2, b2 = params
    M, K = a.shape
    N = w1b.shape[0]
    dw2, db2 = _dw_gemm(nat, dz2, f, w2, b2, st)
    dpre = _mm(nat, dz2, w2b, M, N, K, st, EPI_GELU_GRAD, pre)
    dw1, db1 = _dw_gemm(nat, dpre, a, w1, b1, st)
    da = _mm(nat, dpre, w1b, M, K, N, st) if want_da else None
    return da, dw1, db1, dw2, db2


class _FFNResidualFn(torch.autograd.Function):
    """out = h + W2 gelu(W1 a + b1) + b2: the transformer MLP sub-block as four GEMMs and nothing else.

    Forward stores the GELU pre-activation from the first GEMM's epilogue; backward folds gelu'
    into the epilogue of the dF GEMM (EPI_GELU_GRAD) and both bias gradients into the dW GEMMs'
    column sums, so no elementwise activation-backward pass and no dF intermediate round trip."""

    @staticmethod
    def forward(ctx, a, w1, b1, w2, b2, h):
        nat = native()
        a = a.contiguous()
        if a.dtype != torch.bfloat16:
            a = a.to(torch.bfloat16)
        h = h.contiguous().float()
        w1b, w2b = _w16(w1), _w16(w2)
        f, pre, out = _ffn_fwd(nat, a, w1b, b1, w2b, b2, h, _stream())
        ctx.save_for_backward(a, w1b, w2b, f, pre)
        ctx.params = (w1, b1, w2, b2)
        return out

    @staticmethod
    def backward(ctx, dout):
        a, w1b, w2b, f, pre = ctx.saved_tensors
        grads = _ffn_bwd(native(), _bf16_of(dout), a, w1b, w2b, f, pre, ctx.params, _stream(),
                         ctx.needs_input_grad[0])
        return (*grads, dout)


def ffn_residual(a: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
                 h: torch.Tensor) -> torch.Tensor:
    """h + W2 gelu(W1 a + b1) + b2 (fp32 residual stream; bf16 GEMMs on GPU)."""
    if a.is_cuda:
        return _FFNResidualFn.apply(a, w1, b1, w2, b2, h)
    return h.float() + F.linear(F.gelu(F.linear(a.float(), w1, b1)), w2, b2)


def _ln_fwd(nat, h, w, b, eps, st):
    M, N = h.shape
    a = torch.empty(M, N, dtype=torch.bfloat16, device=h.device)
    mean = torch.empty(M, dtype=torch.float32, device=h.device)
    rstd = torch.empty_like(mean)
    nat.layernorm_fwd(h.data_ptr(), w.data_ptr(), b.data_ptr(), a.data_ptr(), mean.data_ptr(), rstd.data_ptr(), M, N,
                      float(eps), 0, 1, st)
    return a, mean, rstd


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        nat = native()
        x = x.contiguous().float()
        y, mean, rstd = _ln_fwd(nat, x, weight, bias, eps, _stream())
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        nat = native()
        x, weight, mean, rstd = ctx.saved_tensors
        M, N = x.shape
        if _ln_fused_ok(N):
            return (*_ln_bwd(nat, _bf16_of(dy), x, weight, ctx.params[1], mean, rstd), None)
        dy = dy.contiguous().float()
        dx = torch.empty_like(x)
        dw = torch.zeros(N, dtype=torch.float32, device=x.device)
        db = torch.zeros(N, dtype=torch.float32, device=x.device)
        nat.layernorm_bwd(dy.data_ptr(), x.data_ptr(), weight.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                          dx.data_ptr(), dw.data_ptr(), db.data_ptr(), M, N, 0, _stream())
        return dx, dw, db, None


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm over the last dim of a 2-D fp32 input; bf16 output on GPU."""
    if x.is_cuda:
        return _LayerNormFn.apply(x, weight, bias, eps)
    return F.layer_norm(x.float(), (x.shape[-1],), weight, bias, eps)


# ----------------------------------------------------------------------------- fused pre-norm blocks
class _PreNormFFNFn(torch.autograd.Function):
    """h + FFN(LayerNorm(h)) as one autograd node: LN fwd -> GEMM(+b, GELU, keep pre-act) ->
    GEMM(+b, +h residual, fp32).  Backward: the FFN chain above, then ONE LayerNorm-backward
    kernel that also adds the residual-path gradient and emits the bf16 copy the next block's
    GEMMs consume - no autograd adds, no conversions, no per-parameter gradient tensors when bound."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, w1, b1, w2, b2, eps):
        nat = native()
        st = _stream()
        h = h.contiguous().float()
        a, mean, rstd = _ln_fwd(nat, h, ln_w, ln_b, eps, st)
        w1b, w2b = _w16(w1), _w16(w2)
        f, pre, out = _ffn_fwd(nat, a, w1b, b1, w2b, b2, h, st)
        ctx.save_for_backward(h, mean, rstd, a, w1b, w2b, f, pre)
        ctx.params = (ln_w, ln_b, w1, b1, w2, b2)
        return out

    @staticmethod
    def backward(ctx, dout):
        return (*_prenorm_ffn_bwd(dout, ctx.saved_tensors, ctx.params), None)


def _prenorm_ffn_bwd(dout, saved, params):
    """(dh, dln_w, dln_b, dw1, db1, dw2, db2) of h + FFN(LN(h)) from the forward's saved tensors."""
    nat = native()
    st = _stream()
    h, mean, rstd, a, w1b, w2b, f, pre = saved
    ln_w, ln_b = params[:2]
    dout = dout.contiguous().float()
    da, dw1, db1, dw2, db2 = _ffn_bwd(nat, _bf16_of(dout), a, w1b, w2b, f, pre, params[2:], st)
    dh, dlw, dlb = _ln_bwd(nat, da, h, ln_w, ln_b, mean, rstd, dres=dout, want_bf16=True)
    return dh, dlw, dlb, dw1, db1, dw2, db2


class _PreNormAttnFn(torch.autograd.Function):
    """h + Wo Attention(Wqkv LayerNorm(h) + bqkv) + bo as one autograd node (feature-token
    self-attention over T tokens per row, H heads of width D); backward mirrors _PreNormFFNFn."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, wqkv, bqkv, wo, bo, eps, B, H, T):
        nat = native()
        st = _stream()
        h = h.contiguous().float()
        M, dm = h.shape
        D = dm // H
        a, mean, rstd = _ln_fwd(nat, h, ln_w, ln_b, eps, st)
        wqkvb, wob = _w16(wqkv), _w16(wo)
        qkv = torch.empty(M, 3 * dm, dtype=torch.bfloat16, device=h.device)
        nat.gemm_bf16(a.data_ptr(), wqkvb.data_ptr(), qkv.data_ptr(), bqkv.data_ptr(), M, 3 * dm, dm, dm, dm, 3 * dm,
                      0, 1, _EPI[ACT_NONE], 0, 0, 0, st)
        o = torch.empty(M, dm, dtype=torch.bfloat16, device=h.device)
        lse = torch.empty(B * H * T, dtype=torch.float32, device=h.device)
        base = qkv.data_ptr()
        scale = 1.0 / math.sqrt(D)
        nat.attention_fwd(base, base + 2 * dm, base + 4 * dm, o.data_ptr(), lse.data_ptr(), B, H, T, D, 3 * dm, dm,
                          scale, st)
        out = torch.empty(M, dm, dtype=torch.float32, device=h.device)
        nat.gemm_bf16_residual(o.data_ptr(), wob.data_ptr(), out.data_ptr(), bo.data_ptr(), h.data_ptr(), M, dm, dm,
                               st)
        ctx.save_for_backward(h, mean, rstd, a, wqkvb, qkv, o, lse, wob)
        ctx.params = (ln_w, ln_b, wqkv, bqkv, wo, bo)
        ctx.dims = (B, H, T, D, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        return (*_prenorm_attn_bwd(dout, ctx.saved_tensors, ctx.params, ctx.dims), None, None, None, None)


def _prenorm_attn_bwd(dout, saved, params, dims):
    """(dh, dln_w, dln_b, dwqkv, dbqkv, dwo, dbo) of h + Wo MHA(LN(h)) + bo from the saved tensors."""
    nat = native()
    st = _stream()
    h, mean, rstd, a, wqkvb, qkv, o, lse, wob = saved
    ln_w, ln_b, wqkv, bqkv, wo, bo = params
    B, H, T, D, scale = dims
    M, dm = h.shape
    dout = dout.contiguous().float()
    dz = _bf16_of(dout)
    dwo, dbo = _dw_gemm(nat, dz, o, wo, bo, st)
    do = _mm(nat, dz, wob, M, dm, dm, st)
    dqkv = torch.empty_like(qkv)
    base, dbase = qkv.data_ptr(), dqkv.data_ptr()
    nat.attention_bwd(base, base + 2 * dm, base + 4 * dm, o.data_ptr(), do.data_ptr(), lse.data_ptr(), dbase,
                      dbase + 2 * dm, dbase + 4 * dm, B, H, T, D, 3 * dm, dm, scale, st)
    dwqkv, dbqkv = _dw_gemm(nat, dqkv, a, wqkv, bqkv, st)
    da = _mm(nat, dqkv, wqkvb, M, dm, 3 * dm, st)
    dh, dlw, dlb = _ln_bwd(nat, da, h, ln_w, ln_b, mean, rstd, dres=dout, want_bf16=True)
    return dh, dlw, dlb, dwqkv, dbqkv, dwo, dbo


class BatchGather:
    """The step prologue folded into the model's first fused block (csrc/tt_block.hip Gather): the
    autograd engine's captured step hands over, instead of launching ag_step_prologue, where the batch
    comes from (dataset X fp32 [rows][F], int64 row list at a device cursor, int64 labels) and where it
    goes (the step's static x / y - the block writes both, x being its embedding input), plus the step
    counter and the gradient buffer to clear.  ``consumed`` tells the engine a block took it."""

    def __init__(self, X, idx, cursor, stride, n_items, xdst, Y, ydst, step_counter, zero):
        self.values = [X.data_ptr(), idx.data_ptr(), cursor.data_ptr(), int(stride), int(n_items), xdst.data_ptr(),
                       Y.data_ptr(), ydst.data_ptr(), step_counter.data_ptr() if step_counter is not None else 0,
                       zero.data_ptr() if zero is not None else 0, zero.numel() if zero is not None else 0]
        self.xdst = xdst
        self.consumed = False


_BATCH_GATHER: Optional[BatchGather] = None


@contextlib.contextmanager
def fold_batch_gather(spec: BatchGather):
    global _BATCH_GATHER
    prev, _BATCH_GATHER = _BATCH_GATHER, spec
    try:
        yield spec
    finally:
        _BATCH_GATHER = prev


class _TTBlockFn(torch.autograd.Function):
    """A whole pre-norm transformer block (attention sub-block then FFN sub-block) as ONE kernel
    forward (csrc/tt_block.hip: one workgroup per sample, all intermediates in LDS) for the
    TabTransformer shape (64 tokens, d_model 64, 4 heads, FFN 256).  It writes exactly the tensors
    the two unfused nodes save, so the backward is theirs, FFN first."""

    @staticmethod
    def forward(ctx, h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2, eps, B, H, T, pooled=False,
                eE=None, ec=None):
        nat = native()
        st = _stream()
        # eE / ec (the model's first block, with the fused backward): h is the feature matrix x [B, T] and
        # the kernels embed it themselves (x * E + c per token) where they would read the block input
        embed = eE is not None
        h = h.contiguous().float()
        M, dm = (B * T, ln1_w.shape[0]) if embed else h.shape
        FF = w1.shape[0]
        dev = h.device
        wqkvb, wob, w1b, w2b = _w16(wqkv), _w16(wo), _w16(w1), _w16(w2)
        bf, f32 = torch.bfloat16, torch.float32
        a1, a2 = torch.empty(M, dm, dtype=bf, device=dev), torch.empty(M, dm, dtype=bf, device=dev)
        st4 = torch.empty(4, M, dtype=f32, device=dev)  # mean1, rstd1, mean2, rstd2
        # with the fused backward q / k / v are not stored either: tt_block_bwd_kernel recomputes them
        # from a1 with the forward's own MFMAs (bit-identical; 12 MB written and read back per block)
        qkv = torch.empty(0 if _TT_FUSED_BWD and _TT_QKV_RECOMP else M, 3 * dm, dtype=bf, device=dev)
        o = torch.empty(M, dm, dtype=bf, device=dev)
        lse = torch.empty(B * H * T, dtype=f32, device=dev)
        # pooled (the model's last block, training): the kernel writes the token mean [B, dm] the classifier
        # head reads instead of the [B*T, dm] output - which the head read twice (forward and backward)
        h1 = torch.empty(M, dm, dtype=f32, device=dev)
        out = torch.empty(B if pooled else M, dm, dtype=f32, device=dev)
        recomp = _TT_FUSED_BWD
        f = torch.empty(M, FF, dtype=bf, device=dev)
        # with the fused backward the FFN pre-activation is not stored (32 KB per sample written and read
        # back): tt_block_bwd_kernel recomputes it from a2 and W1 (0.3697 -> 0.3632 ms per step,
        # profiles/tt_recompute_pre_ab_r3.log); the unfused backward reads the stored one
        pre = torch.empty(0 if recomp else M, FF, dtype=bf, device=dev)
        wT = torch.empty(2 * FF * dm + 4 * dm * dm, dtype=bf, device=dev)  # W2^T | W1^T | Wo^T | Wqkv^T
        vecs = [t.contiguous() for t in (ln1_w, ln1_b, bqkv, bo, ln2_w, ln2_b, b1, b2)]
        ptrs = [h, vecs[0], vecs[1], wqkvb, vecs[2], wob, vecs[3], vecs[4], vecs[5], w1b, vecs[6], w2b, vecs[7],
                a1, st4[0], st4[1], qkv, o, lse, h1, a2, st4[2], st4[3], f, pre, out, wT]
        scale = 1.0 / math.sqrt(dm // H)
        if _TT_PROF is not None:  # tools/debug/tt_phase_prof.py
            ptrs.append(_tt_prof_buf("fwd", B, dev))
        addrs = [0 if (t is pre and recomp) or (t is out and pooled) or (t is h and embed) or t.numel() == 0
                 else t.data_ptr() for t in ptrs]
        gx = _BATCH_GATHER
        if embed and gx is not None and not gx.consumed and h.data_ptr() == gx.xdst.data_ptr():
            # the step prologue folded in: this launch gathers the batch into h (= the engine's static x)
            nat.tt_block_fwd_gx(addrs, B, T, dm, H, FF, float(eps), scale, out.data_ptr() if pooled else 0,
                                h.data_ptr(), eE.data_ptr(), ec.data_ptr(), gx.values, st)
            gx.consumed = True
        elif pooled or embed:
            em = [t.data_ptr() for t in (h, eE, ec)] if embed else [0, 0, 0]
            nat.tt_block_fwd_ex(addrs, B, T, dm, H, FF, float(eps), scale, out.data_ptr() if pooled else 0, *em, st)
        else:
            nat.tt_block_fwd(addrs, B, T, dm, H, FF, float(eps), scale, st)
        ctx.save_for_backward(h, st4, a1, wqkvb, qkv, o, lse, wob, h1, a2, w1b, w2b, f, pre, wT, vecs[0], vecs[4])
        ctx.embed = (eE, ec) if embed else None
        ctx.params = (ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2)
        ctx.dims = (B, H, T, dm // H, scale)
        ctx.pooled = pooled
        return out

    @staticmethod
    def backward(ctx, dout):
        h, st4, a1, wqkvb, qkv, o, lse, wob, h1, a2, w1b, w2b, f, pre, wT, ln1w, ln2w = ctx.saved_tensors
        p = ctx.params
        B, H, T, D, scale = ctx.dims
        if _TT_FUSED_BWD or pre.numel() == 0 or ctx.pooled or ctx.embed:  # no stored pre-activation: fused
            grads, demb = _tt_block_bwd_fused(dout, h, st4, a1, qkv, o, lse, h1, a2, f, pre, wT, ln1w, ln2w, p, B, H,
                                              T, scale, w1b, pooled=ctx.pooled, embed=ctx.embed, wqkvb=wqkvb)
            if ctx.embed:  # h was the feature matrix: no gradient for it, the embedding's for E / c
                grads = (None,) + tuple(grads[1:])
            return (*grads, None, None, None, None, None, *demb)
        dh1, dl2w, dl2b, dw1, db1, dw2, db2 = _prenorm_ffn_bwd(dout, (h1, st4[2], st4[3], a2, w1b, w2b, f, pre),
                                                               p[6:])
        dh, dl1w, dl1b, dwqkv, dbqkv, dwo, dbo = _prenorm_attn_bwd(
            dh1, (h, st4[0], st4[1], a1, wqkvb, qkv, o, lse, wob), p[:6], ctx.dims)
        return (dh, dl1w, dl1b, dwqkv, dbqkv, dwo, dbo, dl2w, dl2b, dw1, db1, dw2, db2, None, None, None, None, None,
                None, None)


_TT_FUSED_BWD = True
_TT_PROF = None  # {"fwd": [...], "bwd": [...]} of per-workgroup phase timestamp buffers when profiling


def _tt_prof_buf(kind: str, B: int, dev) -> torch.Tensor:
    buf = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    _TT_PROF.setdefault(kind, []).append(buf)
    return buf


_TT_LN_REP = True
_TT_QKV_RECOMP = True
_TT_EMBED_RIDE = True
_TT_LN_WS: Dict[int, torch.Tensor] = {}


def _tt_ln_ws(device: torch.device) -> torch.Tensor:
    """Persistent zeroed workspace of the fused block backward's LayerNorm-gradient replicas:
    16 x 4 x 64 floats + a uint32 ticket (element 4096), left zeroed by every launch.  One
    per device: the block backward kernels of a step run in stream order."""
    ws = _TT_LN_WS.get(device.index)
    if ws is None:
        ws = torch.zeros(16 * 4 * 64 + 4, dtype=torch.float32, device=device)
        _TT_LN_WS[device.index] = ws
    return ws


def _tt_block_bwd_fused(dout, h, st4, a1, qkv, o, lse, h1, a2, f, pre, wT, ln1w, ln2w, params, B, H, T, scale,
                        w1b=None, pooled=False, embed=None, wqkvb=None):
    """Backward of the fused block: ONE kernel for the whole dX chain (csrc/tt_block.hip
    tt_block_bwd_kernel: dF/gelu', W1, LN2, Wo, attention, Wqkv, LN1 per sample) writing the dZ
    operands of the four dW GEMMs, which then run split-K over all rows with the bias gradients
    fused as column sums."""
    nat = native()
    st = _stream()
    ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2 = params
    dout = dout.contiguous().float()
    M, dm = a1.shape  # (h is the feature matrix [B, T] when `embed` = (E, c): the first block)
    FF = w1.shape[0]
    recomp = pre.numel() == 0
    dev, bf = h.device, torch.bfloat16
    dpre = torch.empty(M, FF, dtype=bf, device=dev)
    dh1_16 = torch.empty(M, dm, dtype=bf, device=dev)
    dqkv = torch.empty(M, 3 * dm, dtype=bf, device=dev)
    dh = torch.empty(M, dm, dtype=torch.float32, device=dev)
    dh16 = torch.empty(0 if embed is not None else M, dm, dtype=bf, device=dev)  # embedding block: not needed
    lg = [_grad_dst(t, zero=True) for t in (ln1_w, ln1_b, ln2_w, ln2_b)]
    ptrs = [dout, h, st4[0], st4[1], ln1w, qkv, o, lse, h1, st4[2], st4[3], ln2w, pre, wT,
            dpre, dh1_16, dqkv, dh, dh16] + [g for g, _ in lg]
    addrs = [t.data_ptr() for t in ptrs]
    dout16 = None
    if pooled:  # dout is the head's gradient of the token mean [B, dm]: the kernel broadcasts it (/ T)
        addrs[0] = 0
        dout16 = torch.empty(M, dm, dtype=bf, device=dev)  # bf16(dout), written by the kernel
    if recomp:  # pre-activation recomputed from a2 / W1 / b1 inside the kernel
        addrs[12] = 0
        b1c = b1.detach().contiguous()
        addrs += [a2.data_ptr(), w1b.data_ptr(), b1c.data_ptr()]
    if _TT_PROF is not None:
        addrs.append(_tt_prof_buf("bwd", B, dev).data_ptr())
    if embed is not None:
        addrs[1] = addrs[18] = 0  # the block input is recomputed from x, E, c; no bf16 dh consumer
    em = [t.data_ptr() for t in (h, *embed)] if embed is not None else [0, 0, 0]
    ws = _tt_ln_ws(dev) if _TT_LN_REP else None  # LayerNorm gradients through replicas (csrc LN_REP)
    qr = [0, 0, 0]
    if qkv.numel() == 0:  # q / k / v recomputed from a1 (the forward did not store them)
        bq = bqkv.detach().contiguous()
        qr = [a1.data_ptr(), wqkvb.data_ptr(), bq.data_ptr()]
        addrs[5] = 0
    nat.tt_block_bwd_ex(addrs, B, T, dm, H, FF, scale, dout.data_ptr() if pooled else 0,
                        dout16.data_ptr() if pooled else 0, *em,
                        ws.data_ptr() if ws is not None else 0, ws[4096:].data_ptr() if ws is not None else 0, *qr,
                        st)
    if not pooled:
        dout16 = _bf16_of(dout)
    items = [(dout16, f, w2, b2), (dpre, a2, w1, b1), (dh1_16, o, wo, bo), (dqkv, a1, wqkv, bqkv)]
    b = _BOUND
    direct = b is not None and all(_is_direct(t) for t in (w2, b2, w1, b1, wo, bo, wqkv, bqkv))
    # the first block's embedding gradients ride in the deferred dW launch (queued BEFORE a flush this
    # block may trigger: under DDP its bucket must be complete when the backward returns)
    ride = (embed is not None and direct and b.defer_dw and _TT_EMBED_RIDE
            and all(_is_direct(t) for t in embed))
    if ride:
        _SIDE["embed"] = (h, dh, embed[0].grad, embed[1].grad, B, T, dm)
    if direct and b.defer_dw:
        # accumulate straight into the bound grads at the end of backward, every block in one launch
        _SIDE["deferred"].extend(items)
        b.deferred_blocks += 1
        if b.deferred_blocks in b.flush_at:  # this block closes a bucket group: issue its dW now
            _flush_deferred()
        dw2 = db2 = dw1 = db1 = dwo = dbo = dwqkv = dbqkv = None
    else:
        (dw2, db2), (dw1, db1), (dwo, dbo), (dwqkv, dbqkv) = _dw_gemm_grouped(nat, items, st)
    (dl1w, d1), (dl1b, d2), (dl2w, d3), (dl2b, d4) = lg
    grads = (dh, None if d1 else dl1w, None if d2 else dl1b, dwqkv, dbqkv, dwo, dbo, None if d3 else dl2w,
             None if d4 else dl2b, dw1, db1, dw2, db2)
    if embed is None:
        _remember_bf16(dh, dh16)
        return grads, ()
    if ride:
        return grads, (None, None)
    # the fused embedding's parameter gradients: batch reductions of dh (tt_io.hip embed_bwd_kernel)
    E, c = embed
    dE, dE_direct = _grad_dst(E, zero=True)
    dc, dc_direct = _grad_dst(c, zero=True)
    nat.tt_embed_bwd(h.data_ptr(), dh.data_ptr(), dE.data_ptr(), dc.data_ptr(), B, T, dm, st)
    return grads, (None if dE_direct else dE, None if dc_direct else dc)


def _prenorm_ok(h: torch.Tensor) -> bool:
    return h.is_cuda and _ln_fused_ok(h.shape[1]) and h.shape[1] % 64 == 0


def prenorm_ffn(h, ln_w, ln_b, w1, b1, w2, b2, eps: float = 1e-5):
    """h + W2 gelu(W1 LN(h) + b1) + b2 - one fused autograd node on MI355X."""
    if _prenorm_ok(h):
        return _PreNormFFNFn.apply(h, ln_w, ln_b, w1, b1, w2, b2, eps)
    return ffn_residual(layer_norm(h, ln_w, ln_b, eps), w1, b1, w2, b2, h)


def _tt_block_infer(h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2, eps, B, H, T):
    h = h.contiguous().float()
    dm = h.shape[1]
    out = torch.empty_like(h)
    ws = [_w16(w) for w in (wqkv, wo, w1, w2)]
    ptrs = [h.data_ptr(), ln1_w.data_ptr(), ln1_b.data_ptr(), ws[0].data_ptr(), bqkv.data_ptr(), ws[1].data_ptr(),
            bo.data_ptr(), ln2_w.data_ptr(), ln2_b.data_ptr(), ws[2].data_ptr(), b1.data_ptr(), ws[3].data_ptr(),
            b2.data_ptr()] + [0] * 12 + [out.data_ptr(), 0]
    native().tt_block_fwd(ptrs, B, T, dm, H, w1.shape[0], float(eps), 1.0 / math.sqrt(dm // H), _stream())
    return out


# whole-block TabTransformer kernels (csrc/tt_block.hip) on / off, and their fused backward (tests
# compare them with the per-op autograd nodes by flipping these module flags)
TT_FUSED = True
TT_FUSED_BWD = True


def tt_block_fusable(h: torch.Tensor, H: int, T: int, ffn: int) -> bool:
    """The whole-block fused kernels cover the TabTransformer benchmark shape exactly."""
    global _TT_FUSED_BWD
    _TT_FUSED_BWD = TT_FUSED_BWD
    return h.is_cuda and h.dim() == 2 and h.shape[1] == 64 and H == 4 and T == 64 and ffn == 256 and TT_FUSED


def tt_block(h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2, B: int, H: int, T: int,
             eps: float = 1e-5, pooled: bool = False, embed=None):
    """One pre-norm transformer block: h + MHA(LN1 h), then + FFN(LN2 .) - one fused kernel
    forward on MI355X for the benchmark shape, two fused nodes otherwise.  ``pooled``: return the
    block output's mean over each sample's T tokens, [B, d] (the classifier head's input).
    ``embed`` = (E, c): ``h`` is the feature matrix x [B, T] and the block input is the feature-token
    embedding x * E + c (tt_embed), which the fused kernels compute themselves (first block)."""
    if embed is not None:
        E, c = embed
        x = h
        fuse = (torch.is_grad_enabled() and x.is_cuda and x.dim() == 2 and x.shape[1] == T and E.shape == (T, 64)
                and all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in (E, c)))
        h = None if fuse else tt_embed(x, E, c)
        if fuse and tt_block_fusable(torch.empty(0, 64, device=x.device), H, T, w1.shape[0]) and _TT_FUSED_BWD and \
                all(v.is_contiguous() and v.data_ptr() % 16 == 0 for v in (ln1_w, ln1_b, bqkv, bo, ln2_w, ln2_b, b1, b2)):
            out = _TTBlockFn.apply(x, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2, eps, B, H, T,
                                   False, E, c)
            return out.reshape(B, T, -1).mean(1) if pooled else out
        if h is None:
            h = tt_embed(x, E, c)
    vecs = (ln1_w, ln1_b, bqkv, bo, ln2_w, ln2_b, b1, b2)  # read with 16-byte vector loads
    if tt_block_fusable(h, H, T, w1.shape[0]) and all(v.is_contiguous() and v.data_ptr() % 16 == 0 for v in vecs):
        if not torch.is_grad_enabled():  # validation / serving: the kernel writes only the block output
            out = _tt_block_infer(h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2, eps, B, H, T)
            return out.reshape(B, T, -1).mean(1) if pooled else out
        kp = pooled and _TT_FUSED_BWD  # the kernel pools only for its own (fused) backward
        out = _TTBlockFn.apply(h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2, eps, B, H, T, kp)
        return out.reshape(B, T, -1).mean(1) if pooled and not kp else out
    h = prenorm_attention(h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, B, H, T, eps)
    h = prenorm_ffn(h, ln2_w, ln2_b, w1, b1, w2, b2, eps)
    return h.reshape(B, T, -1).mean(1) if pooled else h


def prenorm_attention(h, ln_w, ln_b, wqkv, bqkv, wo, bo, B: int, H: int, T: int, eps: float = 1e-5):
    """h + Wo MHA(LN(h)) + bo over T feature tokens per row - one fused autograd node on MI355X."""
    if _prenorm_ok(h) and T <= 512 and h.shape[1] // H <= 64:
        return _PreNormAttnFn.apply(h, ln_w, ln_b, wqkv, bqkv, wo, bo, eps, B, H, T)
    a = layer_norm(h, ln_w, ln_b, eps)
    o = attention(linear(a, wqkv, bqkv), B, H, T, h.shape[1] // H)
    return linear_residual(o, wo, bo, h)


class _AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, H, T, D):
        nat = native()
        qkv = qkv.contiguous()
        if qkv.dtype != torch.bfloat16:
            qkv = qkv.to(torch.bfloat16)
        dm = H * D
        o = torch.empty(B * T, dm, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B * H * T, dtype=torch.float32, device=qkv.device)
        scale = 1.0 / math.sqrt(D)
        base = qkv.data_ptr()
        nat.attention_fwd(base, base + 2 * dm, base + 4 * dm, o.data_ptr(), lse.data_ptr(), B, H, T, D, 3 * dm, dm,
                          scale, _stream())
        ctx.dims = (B, H, T, D)
        ctx.save_for_backward(qkv, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        nat = native()
        qkv, o, lse = ctx.saved_tensors
        B, H, T, D = ctx.dims
        dm = H * D
        do = do.contiguous()
        if do.dtype != torch.bfloat16:
            do = do.to(torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        base, dbase = qkv.data_ptr(), dqkv.data_ptr()
        nat.attention_bwd(base, base + 2 * dm, base + 4 * dm, o.data_ptr(), do.data_ptr(), lse.data_ptr(), dbase,
                          dbase + 2 * dm, dbase + 4 * dm, B, H, T, D, 3 * dm, dm, 1.0 / math.sqrt(D), _stream())
        return dqkv, None, None, None, None


def attention(qkv: torch.Tensor, B: int, H: int, T: int, D: int) -> torch.Tensor:
    """Self-attention over T tokens from a packed [B*T, 3*H*D] projection -> [B*T, H*D]."""
    if qkv.is_cuda:
        if T > 512 or D > 64:
            raise ValueError("native attention supports T <= 512 tokens and head dim <= 64")
        return _AttentionFn.apply(qkv, B, H, T, D)
    q, k, v = (t.reshape(B, T, H, D).transpose(1, 2) for t in qkv.float().split(H * D, dim=1))
    o = F.scaled_dot_product_attention(q, k, v)
    return o.transpose(1, 2).reshape(B * T, H * D)


# ----------------------------------------------------------------------------- TabTransformer ends
class _TTEmbedFn(torch.autograd.Function):
    """h[b*F + f, :] = x[b, f] * E[f, :] + c[f, :] (csrc/tt_io.hip); backward = batch reductions."""

    @staticmethod
    def forward(ctx, x, E, c):
        B, F_ = x.shape
        D = E.shape[1]
        x = x.contiguous().float()
        h = torch.empty(B * F_, D, dtype=torch.float32, device=x.device)
        native().tt_embed_fwd(x.data_ptr(), E.contiguous().data_ptr(), c.contiguous().data_ptr(), h.data_ptr(), B,
                              F_, D, _stream())
        ctx.save_for_backward(x)
        ctx.params = (E, c)
        return h

    @staticmethod
    def backward(ctx, dh):
        (x,) = ctx.saved_tensors
        E, c = ctx.params
        B, F_ = x.shape
        dE, dE_direct = _grad_dst(E, zero=True)
        dc, dc_direct = _grad_dst(c, zero=True)
        native().tt_embed_bwd(x.data_ptr(), dh.contiguous().float().data_ptr(), dE.data_ptr(), dc.data_ptr(), B, F_,
                              E.shape[1], _stream())
        return None, None if dE_direct else dE, None if dc_direct else dc


def tt_embed(x: torch.Tensor, E: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """Feature-token embedding [B, F] -> [B*F, D] (native on MI355X for D == 64)."""
    B, F_ = x.shape
    if x.is_cuda and E.shape[1] == 64 and all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in (E, c)):
        return _TTEmbedFn.apply(x, E, c)
    return (x.float()[:, :, None] * E + c).reshape(B * F_, E.shape[1])


_HEAD_SCRATCH: Dict[Optional[int], torch.Tensor] = {}
# superseded scratch buffers stay referenced for the life of the process: a HIP graph captured
# before a regrow still holds the old ticket / partials pointer, and replaying it must never write
# into memory the caching allocator has handed to someone else
_HEAD_SCRATCH_RETIRED: List[torch.Tensor] = []


def _head_scratch(device: torch.device, B: int) -> torch.Tensor:
    """Per-device head-loss scratch: [ticket (uint32 bits, left 0 by every launch) | ceil(B/4) fp32
    partials].  Allocated zeroed by the eager warm-up steps, then reused by the captured step graph
    (one key per device, not per stream: a stream-keyed buffer first met under capture would put its
    zero fill back into every replay).  ONE ticket per device: head forwards must not run
    concurrently on two streams of a device - the engines issue them in stream order on the
    compute stream (a regrow under an active capture is refused for the same reason)."""
    key = device.index
    n = 1 + (B + 3) // 4
    buf = _HEAD_SCRATCH.get(key)
    if buf is None or buf.numel() < n:
        if buf is not None and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("tt head scratch must be sized by an eager step before graph capture")
        if buf is not None:
            _HEAD_SCRATCH_RETIRED.append(buf)
        buf = torch.zeros(max(n, 1 + 128), dtype=torch.float32, device=device)
        _HEAD_SCRATCH[key] = buf
    return buf


# Set by the autograd engine around a training step whose loss.backward() seed is exactly 1 (its
# persistent ones seed, trainer/engines.py _backward): the classifier head then computes its backward in
# the forward launch (dct_tt_head_fused) and the backward only hands the results over - one launch less
# per step.  Anywhere else (a scaled loss, a user's own backward) the head keeps its two launches.
_UNIT_LOSS_SEED = False


@contextlib.contextmanager
def unit_loss_seed():
    global _UNIT_LOSS_SEED
    prev, _UNIT_LOSS_SEED = _UNIT_LOSS_SEED, True
    try:
        yield
    finally:
        _UNIT_LOSS_SEED = prev


class _TTHeadLossFn(torch.autograd.Function):
    """mean_b CE(Linear(LN(mean_t h[b, t, :])), y_b) in one kernel; the backward kernel recomputes the
    per-sample chain and writes dh (fp32 + the bf16 copy the last block's dW GEMM consumes).  Under
    unit_loss_seed() a training forward runs both in one launch (the backward returns its results)."""

    @staticmethod
    def forward(ctx, h, y, ln_w, ln_b, W, bias, B, T, eps, root=False):
        h = h.contiguous().float()
        y = y.contiguous().long()
        vec = [t.contiguous() for t in (ln_w, ln_b, W, bias)]
        loss = torch.empty((), dtype=torch.float32, device=h.device)  # stored by the kernel's last block
        scratch = _head_scratch(h.device, B)
        ctx.params = (ln_w, ln_b, W, bias)
        ctx.dims = (B, T, eps)
        ctx.fused = None
        if root and _UNIT_LOSS_SEED and ctx.needs_input_grad[0]:
            dh = torch.empty_like(h)
            dh16 = torch.empty(h.shape, dtype=torch.bfloat16, device=h.device)
            gs = [_grad_dst(p, zero=True) for p in ctx.params]
            native().tt_head_fused([h.data_ptr(), y.data_ptr()] + [t.data_ptr() for t in vec]
                                   + [loss.data_ptr(), scratch.data_ptr() + 4, scratch.data_ptr(), dh.data_ptr(),
                                      dh16.data_ptr()] + [g.data_ptr() for g, _ in gs], B, T,
                                   h.shape[1], W.shape[0], float(eps), _stream())
            ctx.fused = (dh, dh16, gs)
            return loss
        native().tt_head_fwd([h.data_ptr(), y.data_ptr()] + [t.data_ptr() for t in vec]
                             + [loss.data_ptr(), scratch.data_ptr() + 4, scratch.data_ptr()], B, T,
                             h.shape[1], W.shape[0], float(eps), _stream())
        ctx.save_for_backward(h, y, *vec)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        if ctx.fused is not None:  # computed by the forward launch for dloss = 1 (unit_loss_seed)
            dh, dh16, gs = ctx.fused
            ctx.fused = None
            _remember_bf16(dh, dh16)
            return (dh, None, *[None if direct else g for g, direct in gs], None, None, None, None)
        h, y, lw, lb, Wc, bc = ctx.saved_tensors
        B, T, eps = ctx.dims
        dh = torch.empty_like(h)
        dh16 = torch.empty(h.shape, dtype=torch.bfloat16, device=h.device)
        gs = [_grad_dst(p, zero=True) for p in ctx.params]
        dloss = dloss.contiguous().float()
        ptrs = [h, y, lw, lb, Wc, bc, dloss, dh, dh16] + [g for g, _ in gs]
        native().tt_head_bwd([t.data_ptr() for t in ptrs], B, T, h.shape[1], Wc.shape[0], float(eps), _stream())
        _remember_bf16(dh, dh16)
        return (dh, None, *[None if direct else g for g, direct in gs], None, None, None, None)


def tt_head_fusable(h: torch.Tensor, num_classes: int) -> bool:
    return h.is_cuda and h.shape[1] == 64 and 1 <= num_classes <= 8


def tt_head_loss(h, y, B: int, T: int, ln_w, ln_b, W, bias, eps: float = 1e-5, root: bool = False):
    """Mean cross-entropy of the pooled-token classifier head (LN -> Linear) - one kernel each way.
    ``root``: the caller returns this loss unscaled as the step's backward root, so under
    unit_loss_seed() (backward seed exactly 1) the forward launch may compute the backward as well."""
    if tt_head_fusable(h, W.shape[0]):
        return _TTHeadLossFn.apply(h, y, ln_w, ln_b, W, bias, B, T, eps, root)
    pooled = h.reshape(B, T, h.shape[1]).mean(1)
    z = layer_norm(pooled, ln_w, ln_b, eps)
    return F.cross_entropy(linear(z, W, bias).float(), y)
