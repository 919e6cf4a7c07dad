"""dxa — an MI355X-native streaming data-pipeline engine (Data Accelerator capabilities on PyTorch-ROCm, hand-written
gfx950 HIP kernels and RCCL over xGMI).  See README.md for the layer map."""
__version__ = "0.1.0"
