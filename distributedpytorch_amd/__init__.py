"""distributedpytorch_amd - MI355X-native (gfx950 / CDNA4) distributed UNet training framework.

Capability parity with notnitsuj/DistributedPyTorch (single GPU, DataParallel,
DistributedDataParallel, pipeline model parallelism of a 4-level UNet with BCE - log Dice loss),
re-designed for MI355X: hand-written HIP kernels (MFMA implicit-GEMM convs, fused loss, fused
Adam), RCCL over xGMI for gradient buckets and pipeline send/recv, one process per GPU.
"""
__version__ = "0.1.0"

from .models.unet import UNet, UNetConfig, build_model  # noqa: E402,F401
from .loss import Loss  # noqa: E402,F401
