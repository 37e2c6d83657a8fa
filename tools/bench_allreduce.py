#!/usr/bin/env python3
"""All-reduce busBW / latency sweep (dct_amd.parallel.commbench); one rank per GPU:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/bench_allreduce.py --max-bytes 268435456
    python tools/bench_allreduce.py                      # W = 1: RCCL launch latency only
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402,F401
from dct_amd.parallel.commbench import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
