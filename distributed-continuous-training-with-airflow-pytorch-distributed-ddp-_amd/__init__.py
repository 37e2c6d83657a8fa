"""dct_amd - MI355X-native distributed continuous-training framework.

Capabilities of the reference pipeline (Airflow -> Spark ETL -> Lightning DDP training ->
MLflow -> Azure ML rollout), rebuilt around PyTorch-ROCm, hand-written HIP/CDNA4 kernels and
RCCL over xGMI.  Import as ``import dct_amd`` (see ``dct_amd.py`` at the repository root).
"""
__version__ = "0.1.0"

from .config import PipelineConfig, default_config  # noqa: F401
