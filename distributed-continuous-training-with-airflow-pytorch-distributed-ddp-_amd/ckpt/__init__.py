from .callbacks import ModelCheckpoint  # noqa: F401
from .lightning_io import (CHECKPOINT_KEYS, build_checkpoint, elastic_restart_count, load_checkpoint,  # noqa: F401
                          resume_checkpoint, save_checkpoint)
