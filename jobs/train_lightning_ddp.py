"""Reference-named training entry point (reference: jobs/train_lightning_ddp.py, run as
``python3 /workspace/jobs/train_lightning_ddp.py`` with no arguments on every rank).

Honours the reference's env contract (``WORLD_SIZE``, ``NODE_RANK``, ``MASTER_ADDR``,
``MASTER_PORT``, ``MLFLOW_TRACKING_URI``) as well as torchrun's, with the reference defaults
(data ``/workspace/data/processed``, checkpoints ``/workspace/data/models``, batch 4, lr 0.01,
10 epochs).  All logic lives in ``jobs/train_ddp.py``; extra flags are forwarded.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from train_ddp import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
