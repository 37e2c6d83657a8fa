"""Split + sharding with the exact index semantics of the reference's data path.

* ``seeded_random_split``: ``torch.utils.data.random_split`` after ``seed_everything(42)``
  (train_lightning_ddp.py:14,117-119) - ``randperm(n)`` from a generator seeded with the
  global seed, first ``int(0.8 n)`` indices train, rest val.
* ``distributed_indices``: what Lightning's DDP strategy injects [lib] -
  ``DistributedSampler(num_replicas=W, rank=r, shuffle, seed=PL_GLOBAL_SEED)``:
  ``randperm(n, generator(seed + epoch))`` when shuffling, padded by wrapping to
  ``ceil(n / W) * W``, then ``indices[rank::W]``.  The permutation is produced with torch's
  CPU generator (so shards match torch bit-for-bit) and uploaded once per epoch; the gather
  itself runs on the device.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch


def seeded_random_split(n: int, train_fraction: float = 0.8, seed: int = 42,
                        generator: Optional[torch.Generator] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    train_size = int(train_fraction * n)
    g = generator
    if g is None:
        g = torch.Generator()
        g.manual_seed(seed)
    perm = torch.randperm(n, generator=g)
    return perm[:train_size], perm[train_size:]


def distributed_indices(n: int, world_size: int = 1, rank: int = 0, shuffle: bool = True,
                        seed: int = 42, epoch: int = 0, drop_last: bool = False) -> torch.Tensor:
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError(f"invalid rank {rank} for world size {world_size}")
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g)
    else:
        indices = torch.arange(n)
    if drop_last and n % world_size != 0:
        num_samples = math.ceil((n - world_size) / world_size)
    else:
        num_samples = math.ceil(n / world_size)
    total = num_samples * world_size
    if not drop_last:
        pad = total - n
        if pad > 0:
            if pad <= n:
                indices = torch.cat([indices, indices[:pad]])
            else:
                reps = math.ceil(pad / n)
                indices = torch.cat([indices, indices.repeat(reps)[:pad]])
    else:
        indices = indices[:total]
    assert len(indices) == total
    return indices[rank:total:world_size]


def batches(indices: torch.Tensor, batch_size: int, drop_last: bool = False) -> List[torch.Tensor]:
    out = []
    for s in range(0, len(indices), batch_size):
        b = indices[s : s + batch_size]
        if drop_last and len(b) < batch_size:
            break
        out.append(b)
    return out


def num_batches(n_local: int, batch_size: int, drop_last: bool = False) -> int:
    return n_local // batch_size if drop_last else math.ceil(n_local / batch_size)
