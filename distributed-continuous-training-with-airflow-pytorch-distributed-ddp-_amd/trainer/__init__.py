from .module import TrainModule  # noqa: F401
from .trainer import DDPStrategy, Trainer, seed_everything  # noqa: F401
