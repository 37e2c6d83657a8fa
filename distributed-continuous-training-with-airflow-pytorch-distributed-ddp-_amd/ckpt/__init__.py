from .callbacks import ModelCheckpoint  # noqa: F401
from .lightning_io import CHECKPOINT_KEYS, build_checkpoint, load_checkpoint, save_checkpoint  # noqa: F401
