"""Autograd functions over the native HIP kernels (bf16 activations, fp32 master weights).

Used by the transformer-style models (models/tabtransformer.py) on MI355X:
  * ``linear``     - MFMA GEMM forward with fused bias / ReLU / GELU epilogue; backward = two
                     GEMMs (dX = dZ W, dW = dZ^T X with the bias gradient fused as a column sum)
                     and one elementwise activation-derivative pass when needed;
  * ``layer_norm`` - one wave per row, fp32 statistics (fwd) / fused dX, dgamma, dbeta (bwd);
  * ``attention``  - fused feature-token attention over a packed QKV projection (online softmax
                     forward, recompute backward).
On CPU (the gloo plumbing config) the same functions fall back to plain torch ops; on a GPU the
native module is required (``native()`` raises if it is missing - no silent fallback).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ._native import native

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2
_EPI = {ACT_NONE: 1, ACT_RELU: 2, ACT_GELU: 3}  # EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_GELU


def _stream():
    return torch.cuda.current_stream().cuda_stream


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act):
        nat = native()
        x = x.contiguous()
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        M, K = x.shape
        N = weight.shape[0]
        wb = weight.detach().to(torch.bfloat16).contiguous()
        y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        pre = torch.empty_like(y) if act == ACT_GELU else None
        nat.gemm_bf16(x.data_ptr(), wb.data_ptr(), y.data_ptr(), bias.data_ptr(), M, N, K, K, K, N, 0, 1, _EPI[act], 0,
                      0, pre.data_ptr() if pre is not None else 0, _stream())
        ctx.act = act
        ctx.save_for_backward(x, wb, y if act == ACT_RELU else pre)
        return y

    @staticmethod
    def backward(ctx, dy):
        nat = native()
        x, wb, aux = ctx.saved_tensors
        act = ctx.act
        dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        M, K = x.shape
        N = wb.shape[0]
        st = _stream()
        db = torch.zeros(N, dtype=torch.float32, device=x.device)
        if act == ACT_NONE:
            dz = dy
            colsum = db.data_ptr()
        else:  # dZ = dY * act'(.) and db in one pass
            dz = torch.empty_like(dy)
            nat.bias_act_bwd(dy.data_ptr(), aux.data_ptr(), dz.data_ptr(), db.data_ptr(), M, N, N, act, 1, st)
            colsum = 0
        dw = torch.empty(N, K, dtype=torch.float32, device=x.device)
        nat.gemm_bf16_ex(dz.data_ptr(), x.data_ptr(), dw.data_ptr(), 0, N, K, M, N, K, K, 1, 0, 0, 1, 0, 0, colsum, st)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=x.device)
            nat.gemm_bf16(dz.data_ptr(), wb.data_ptr(), dx.data_ptr(), 0, M, K, N, N, K, K, 0, 0, 0, 0, 0, 0, st)
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
        wb = weight.detach().to(torch.bfloat16).contiguous()
        out = torch.empty(M, N, dtype=torch.float32, device=x.device)
        nat.gemm_bf16_residual(x.data_ptr(), wb.data_ptr(), out.data_ptr(), bias.data_ptr(), h.data_ptr(), M, N, K,
                               _stream())
        ctx.save_for_backward(x, wb)
        return out

    @staticmethod
    def backward(ctx, dout):
        nat = native()
        x, wb = ctx.saved_tensors
        M, K = x.shape
        N = wb.shape[0]
        st = _stream()
        dz = dout.contiguous().to(torch.bfloat16)
        db = torch.zeros(N, dtype=torch.float32, device=x.device)
        dw = torch.empty(N, K, dtype=torch.float32, device=x.device)
        nat.gemm_bf16_ex(dz.data_ptr(), x.data_ptr(), dw.data_ptr(), 0, N, K, M, N, K, K, 1, 0, 0, 1, 0, 0,
                         db.data_ptr(), st)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=x.device)
            nat.gemm_bf16(dz.data_ptr(), wb.data_ptr(), dx.data_ptr(), 0, M, K, N, N, K, K, 0, 0, 0, 0, 0, 0, st)
        return dx, dw, db, dout


def linear_residual(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """h + x W^T + b (fp32): on GPU one GEMM with the residual folded into its epilogue."""
    if x.is_cuda:
        return _LinearResidualFn.apply(x, weight, bias, h)
    return h.float() + F.linear(x.float(), weight, bias)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        nat = native()
        x = x.contiguous().float()
        M, N = x.shape
        y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        nat.layernorm_fwd(x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(), mean.data_ptr(),
                          rstd.data_ptr(), M, N, float(eps), 0, 1, _stream())
        ctx.save_for_backward(x, weight, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        nat = native()
        x, weight, mean, rstd = ctx.saved_tensors
        M, N = x.shape
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
