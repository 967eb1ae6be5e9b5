"""unetseg_hip: MI355X-native (gfx950) runtime of the U-Net segmentation training hot path.

Python host over the C ABI of libunetseg_hip.so (include/unetseg_hip.h): hand-written HIP kernels
for implicit-GEMM MFMA convolutions, BatchNorm, pooling, upsampling, attention gates, losses,
metrics and Adam.  PyTorch-ROCm provides device memory, streams and torch.distributed (RCCL).
"""
from .lib import DT_BF16, DT_F32, HipUnavailable, LIB_PATH, exported_symbols, load  # noqa: F401

__all__ = ["DT_BF16", "DT_F32", "HipUnavailable", "LIB_PATH", "exported_symbols", "load"]
