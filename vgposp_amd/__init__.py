"""vgposp_amd — MI355X-native hot path of DL-WG/VGPosp (GP kernel assembly -> fp64 Cholesky ->
GP / VGP fit-and-predict -> greedy mutual-information sensor placement).

Host Python mirrors the reference's own surface (``placement_algorithm2``, ``gp_functions``, the
TFP-shaped ``GaussianProcess`` / ``GaussianProcessRegressionModel`` / ``VariationalGaussianProcess``)
and drives hand-written HIP kernels for gfx950 in ``libvgposp.so`` through the C-ABI of
``include/vgposp.h``.  PyTorch-ROCm only holds device memory and streams.
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401  (ctypes binding; loads lazily)
