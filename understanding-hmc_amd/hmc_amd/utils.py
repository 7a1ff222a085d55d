"""Helpers with the reference `utils.py` names (utils.py:77-218).

`start_pts` and `normal_lnL` are the host helpers the drivers call to build
their inputs (they stay NumPy/SciPy, as in the reference).  `convergence_stats`
(split-chain R-hat and ESS, utils.py:77-159) runs on the GPU through the
diagnostics kernels of libhmc.so (diagnostics.py); NUTS bookkeeping helpers are
restated as integer bit logic (the GPU NUTS kernel uses the same closed forms).
"""
import numpy as np
from scipy.stats import multivariate_normal

from .diagnostics import convergence_stats, per_dim_mean_std, variogram  # noqa: F401


def start_pts(q0, cov0, size):
    """utils.py:204-209 (host draw from the global legacy RNG, exactly as the reference)."""
    return np.random.multivariate_normal(q0, cov0, size=size)


START_ITERATION = 0x7FFFFFFF   # Philox iteration word reserved for start points (no run reaches it)


def start_pts_device(seed, chain0, n, D, scale=np.sqrt(2.0), device=None):
    """utils.py:204-209 for many chains on the device: q_start[c] = scale * z, z ~ N(0, I_D), keyed
    by (seed, GLOBAL chain id chain0 + c) through the kernels' Philox4x32-10 + Box-Muller (C-ABI
    hmc_rng_normals, iteration word START_ITERATION), so a chain starts from the same point
    whichever shard or GPU count holds it.  Returns an (n, D) float64 device tensor."""
    import torch
    from . import _lib as H
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    npairs = (int(D) + 1) // 2
    out = torch.empty((int(n), 2 * npairs), dtype=torch.float64, device=dev)
    H.check(H.lib().hmc_rng_normals(int(seed), int(chain0), int(n), START_ITERATION, npairs, H.ptr(out),
                                    torch.cuda.current_stream(dev).cuda_stream), "hmc_rng_normals")
    return (out[:, :D] * float(scale)).contiguous()


def normal_lnL(q, q0, cov0):
    """utils.py:213-218."""
    return multivariate_normal.logpdf(q, mean=q0, cov=cov0)


def check_points(m):
    """utils.py:246-283 in closed form: for even m, the first point of every aligned
    power-of-two sub-tree (size >= 2) ending at m."""
    assert (m % 2) == 0
    r = int(m)
    while (r & (r - 1)) != 0 and r > 2:
        r -= 1 << (r.bit_length() - 1)
    pts = [m - r + 1]
    half = r
    while half > 2:
        half >>= 1
        pts.append(pts[-1] + half)
    return np.asarray(pts)


def release_fast(m, l):
    """utils.py:367-385."""
    r_m, r_l = int(m), int(l)
    while (r_m & (r_m - 1)) != 0 and r_m > 4:
        top = 1 << (r_m.bit_length() - 1)
        r_m -= top
        r_l -= top
    return (r_m >= 4) and (r_l > 1)


release = release_fast   # utils.py:286-304 implements the same rule (with an assert)
