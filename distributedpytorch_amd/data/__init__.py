"""Datasets: synthetic segmentation (GPU-resident capable) and the Carvana folder layout.

Parity target: reference ``utils/dataloading.py:12-78`` for the folder dataset and
``utils/train_utils.py:27-42`` for the split / loaders (one seeded split everywhere, quirk A8 fixed).
"""
from .synthetic import SyntheticSegmentation, synthetic_batch
from .folder import BasicDataset, CarvanaDataset
from .loaders import split_dataset, build_loaders, DeviceBatcher
from .device import DeviceSyntheticSegmentation, DeviceLoader, device_loaders

__all__ = [
    "SyntheticSegmentation", "synthetic_batch", "BasicDataset", "CarvanaDataset",
    "split_dataset", "build_loaders", "DeviceBatcher",
    "DeviceSyntheticSegmentation", "DeviceLoader", "device_loaders",
]
