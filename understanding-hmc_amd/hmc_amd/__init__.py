"""hmc_amd — MI355X-native many-chain HMC (the samplers.py hot path of
jaekor91/understanding-HMC) behind the reference's sampler-class surface.

    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.utils import start_pts, normal_lnL, convergence_stats

The compute path is libhmc.so (HIP, gfx950) through its C ABI (include/hmc.h).
"""
__version__ = "0.1.0"
