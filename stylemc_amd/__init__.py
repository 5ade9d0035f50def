"""stylemc_amd -- MI355X-native (gfx950) implementation of StyleMC's find_direction hot path.

Host code is Python on PyTorch-ROCm mirroring the reference's interfaces; the compute runs in the
hand-written HIP kernels of ``libstylemc_hip.so`` (C ABI: include/stylemc_hip.h).
"""
__version__ = "0.1.0"
