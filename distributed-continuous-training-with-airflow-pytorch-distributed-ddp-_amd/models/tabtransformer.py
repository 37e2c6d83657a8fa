"""TabTransformer-style model over feature tokens (BASELINE.json config 5).

Each numeric feature f of a row becomes a token ``x_f * E_f + c_f`` (d_model wide); L pre-norm
transformer blocks (LayerNorm -> packed QKV -> feature-token attention -> out projection ->
residual; LayerNorm -> GELU MLP -> residual) mix the tokens; the mean token goes through a
final LayerNorm and a linear head.  On MI355X every GEMM / LayerNorm / attention is a native
HIP kernel (ops/nn.py) with bf16 activations on an fp32 residual stream, and each pre-norm sub-block
is ONE fused autograd node (prenorm_attention / prenorm_ffn) - at the benchmark shape the whole
block's forward is one kernel (ops/nn.py tt_block, csrc/tt_block.hip); on CPU the same module runs
plain torch ops.  Training contract = the reference LightningModule's (training_step logs
``train_loss``; validation_step logs ``val_loss`` / ``val_acc``; Adam).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.nn import layer_norm, linear, tt_block, tt_embed, tt_head_loss
from ..trainer.module import TrainModule


# the last block hands the classifier head the token mean (ops/nn.py tt_block(pooled=True)); False: the
# head pools the last block's full output itself (A/B: tools/tt_pooled_head_ab.py)
POOLED_HEAD = True
# the first block computes the feature-token embedding where it reads its input (tt_block(embed=...));
# False: a separate embedding kernel writes the [B*F, d] input (A/B: tools/tt_pooled_head_ab.py)
FUSED_EMBED = True


class _Block(nn.Module):
    def __init__(self, d: int, heads: int, ffn_mult: int):
        super().__init__()
        self.heads = heads
        self.ln1_w, self.ln1_b = nn.Parameter(torch.ones(d)), nn.Parameter(torch.zeros(d))
        self.qkv = nn.Linear(d, 3 * d)
        self.proj = nn.Linear(d, d)
        self.ln2_w, self.ln2_b = nn.Parameter(torch.ones(d)), nn.Parameter(torch.zeros(d))
        self.fc1 = nn.Linear(d, ffn_mult * d)
        self.fc2 = nn.Linear(ffn_mult * d, d)

    def forward(self, h: torch.Tensor, B: int, T: int, pooled: bool = False, embed=None) -> torch.Tensor:
        return tt_block(h, self.ln1_w, self.ln1_b, self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias,
                        self.ln2_w, self.ln2_b, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias,
                        B, self.heads, T, pooled=pooled, embed=embed)


class TabTransformer(TrainModule):
    # its fused blocks may defer their weight-gradient GEMMs to one grouped launch after backward
    # (ops/nn.py tt_block): a bucket reducer must then launch at finalize, not from the hooks
    uses_fused_blocks = True

    def __init__(self, num_features: int = 64, d_model: int = 64, heads: int = 4, layers: int = 4, ffn_mult: int = 4,
                 num_classes: int = 2, lr: float = 1e-3):
        super().__init__()
        self.save_hyperparameters()
        if d_model % heads:
            raise ValueError("d_model must be divisible by heads")
        self.F, self.d, self.lr = num_features, d_model, lr
        self.feat_w = nn.Parameter(torch.randn(num_features, d_model) / math.sqrt(d_model))
        self.feat_b = nn.Parameter(torch.zeros(num_features, d_model))
        self.blocks = nn.ModuleList([_Block(d_model, heads, ffn_mult) for _ in range(layers)])
        self.ln_w, self.ln_b = nn.Parameter(torch.ones(d_model)), nn.Parameter(torch.zeros(d_model))
        self.head = nn.Linear(d_model, num_classes)

    @property
    def folds_batch_gather(self) -> bool:
        """The first block embeds the features itself, so it can also gather them (ops/nn.py
        fold_batch_gather: the autograd engine's captured step then has no prologue launch)."""
        return FUSED_EMBED and len(self.blocks) > 0

    def _trunk(self, x: torch.Tensor, pooled: bool = False) -> torch.Tensor:
        """Token embedding + the blocks: [B*F, d], or with ``pooled`` the last block's output averaged
        over each sample's F tokens, [B, d] (on MI355X the last block kernel writes only that)."""
        B = x.shape[0]
        if not FUSED_EMBED or len(self.blocks) == 0:
            h = tt_embed(x, self.feat_w, self.feat_b)
            for i, blk in enumerate(self.blocks):
                h = blk(h, B, self.F, pooled=pooled and i == len(self.blocks) - 1)
            return h
        # the first block embeds the features itself (ops/nn.py tt_block(embed=...)): the [B*F, d] block
        # input is never written to or read from HBM in the fused training step
        h = x
        for i, blk in enumerate(self.blocks):
            h = blk(h, B, self.F, pooled=pooled and i == len(self.blocks) - 1,
                    embed=(self.feat_w, self.feat_b) if i == 0 else None)
        return h

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0]
        pooled = self._trunk(x).reshape(B, self.F, self.d).mean(1)
        z = layer_norm(pooled, self.ln_w, self.ln_b)
        return linear(z, self.head.weight, self.head.bias).float()

    def training_step(self, batch, batch_idx):
        x, y = batch
        # pooled LN -> Linear -> mean CE as one kernel each way on MI355X (ops/nn.py tt_head_loss)
        # (the head consumes the pooled tokens: the last block hands over [B, d], not [B*F, d])
        # (root: this loss is returned unscaled - the engine's backward seed reaches the head as exactly 1)
        if POOLED_HEAD:
            loss = tt_head_loss(self._trunk(x, pooled=True), y, x.shape[0], 1, self.ln_w, self.ln_b, self.head.weight,
                                self.head.bias, root=True)
        else:
            loss = tt_head_loss(self._trunk(x), y, x.shape[0], self.F, self.ln_w, self.ln_b, self.head.weight,
                                self.head.bias, root=True)
        self.log("train_loss", loss, sync_dist=True)
        return loss

    def validation_step(self, batch, batch_idx):
        x, y = batch
        logits = self(x)
        loss = F.cross_entropy(logits, y)
        acc = (logits.argmax(1) == y).float().mean()
        self.log("val_loss", loss, sync_dist=True, prog_bar=True)
        self.log("val_acc", acc, sync_dist=True, prog_bar=True)
        return loss

    def ddp_block_groups(self):
        """Blocks grouped for data-parallel gradient buckets, in backward order: the upper half of
        the blocks (with the head / final LayerNorm, whose gradients come first), then the rest
        (with the token embedding).  The engine aligns its DDP buckets with these groups and
        issues each group's deferred dW GEMMs as one grouped launch inside the backward of the
        group's last block, so the first bucket's all-reduce runs under the remaining backward
        (trainer/engines.py AutogradEngine, ops/nn.py bound_params).  None: one group."""
        L = len(self.blocks)
        if L < 2:
            return None
        hi = L - L // 2
        return [list(range(L - 1, L - 1 - hi, -1)), list(range(L - 1 - hi, -1, -1))]

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr)
