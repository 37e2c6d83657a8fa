from .dist import DistContext, init_distributed, init_native_comm, resolve_env, shutdown  # noqa: F401
from .reducer import BucketPlan, NativeBucketReducer, TorchBucketReducer, plan_buckets  # noqa: F401
