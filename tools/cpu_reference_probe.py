#!/usr/bin/env python3
"""Plain-PyTorch CPU stand-in of the reference training step (BASELINE.md "Local probe").

Mirrors jobs/train_lightning_ddp.py's hot loop without Lightning (which only adds overhead):
a map-style Dataset with per-sample __getitem__ (:49), DataLoader(batch_size=4, shuffle=True,
num_workers=0) collate (:122), Linear/ReLU/Dropout(0.2) MLP (:57-62), F.cross_entropy (:69),
loss.backward(), Adam(lr=0.01) (:88).  World size 1.  Prints samples/s for the reference
5-64-2 and BASELINE's 3-layer 128-h variant - the denominators of bench.py's vs_baseline.

    python tools/cpu_reference_probe.py [steps]
"""
import json
import sys
import time

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset


class Rows(Dataset):
    def __init__(self, X, Y):
        self.X, self.Y = X, Y

    def __len__(self):
        return len(self.Y)

    def __getitem__(self, i):
        return self.X[i], self.Y[i]


def net(hidden):
    layers, d = [], 5
    for h in hidden:
        layers += [torch.nn.Linear(d, h), torch.nn.ReLU(), torch.nn.Dropout(0.2)]
        d = h
    layers.append(torch.nn.Linear(d, 2))
    return torch.nn.Sequential(*layers)


def probe(hidden, steps, warmup=200):
    torch.manual_seed(42)
    n = (steps + warmup) * 4
    ds = Rows(torch.randn(n, 5), torch.randint(0, 2, (n,)))
    model = net(hidden)
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    it = iter(DataLoader(ds, batch_size=4, shuffle=True, num_workers=0))
    t0 = None
    for s in range(steps + warmup):
        if s == warmup:
            t0 = time.perf_counter()
        x, y = next(it)
        loss = F.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
    dt = time.perf_counter() - t0
    return steps * 4 / dt, dt / steps * 1e6


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    torch.set_num_threads(int(torch.get_num_threads()))
    out = {}
    for name, hidden in (("weather 5-64-2", [64]), ("weather-mlp-3x128 5-128-128-2", [128, 128])):
        sps, us = probe(hidden, steps)
        out[name] = {"samples_per_s": round(sps, 1), "us_per_step": round(us, 1)}
    print(json.dumps({"torch": torch.__version__, "threads": torch.get_num_threads(), "steps": steps, **out}))


if __name__ == "__main__":
    main()
