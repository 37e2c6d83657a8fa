from .dataset import DeviceTensorDataset, TensorPairDataset, WeatherDataset, dataset_tensors
from .sampler import batches, distributed_indices, num_batches, seeded_random_split

__all__ = [
    "WeatherDataset", "TensorPairDataset", "DeviceTensorDataset", "dataset_tensors",
    "seeded_random_split", "distributed_indices", "batches", "num_batches",
]
