from .logger import InMemoryLogger, MLFlowLogger  # noqa: F401
from .mlflow_client import FileStore, MlflowClient, RestStore  # noqa: F401
