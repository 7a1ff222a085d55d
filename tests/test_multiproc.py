"""Multi-rank (N>1) path on the CPU: world_size-2 `gloo` process groups.

Chains shard across ranks by global chain id; the only exchange is the all-reduce of the
split-chain sums inside the diagnostics (hmc_amd.diagnostics.combine_split_stats, the same
code the GPUs run over RCCL).  Each rank here holds half of the chains of a fixed q_chain and
its per-chain moments / variogram lag sums (restated with NumPy as the device kernels would
produce them); the combined R-hat / ESS must equal the single-process oracle on all chains.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from oracle import hmc_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_stats(q, n, T):
    """What a rank's device kernels produce for its chains q (N, 2n+, D): split means/stds
    (2N, D) and variogram lag sums (T, D) over its split chains."""
    halves = [q[:, h * n:(h + 1) * n, :] for h in (0, 1)]
    xs = np.stack(halves, axis=1).reshape(-1, n, q.shape[2])           # (2N, n, D) chain-major
    mean = xs.mean(axis=1)
    std = xs.std(axis=1, ddof=1)
    v = np.stack([((xs[:, t:, :] - xs[:, :-t, :]) ** 2).sum(axis=(0, 1)) for t in range(1, T + 1)])
    return mean, std, v


def _worker(rank, world, port, q_all, T, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hmc_amd.diagnostics import combine_split_stats
        N = q_all.shape[0]
        lo, hi = rank * N // world, (rank + 1) * N // world                # contiguous chain shard
        n = q_all.shape[1] // 2
        mean, std, v = _rank_stats(q_all[lo:hi], n, T)
        R, neff = combine_split_stats(torch.from_numpy(mean), torch.from_numpy(std), torch.from_numpy(v), n,
                                      group=dist.group.WORLD)
        out[rank] = (R, neff)
    finally:
        dist.destroy_process_group()


def _run(q_all, T, world=2):
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_worker, args=(world, _free_port(), q_all, T, out), nprocs=world, join=True)
    return dict(out)


def _ar1(N, L, D, rho, seed):
    rs = np.random.RandomState(seed)
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D))
    for t in range(1, L):
        x[:, t] = rho * x[:, t - 1] + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    return x


@pytest.mark.parametrize("rho,T", [(0.3, 32), (0.0, 8), (-0.2, 16)])
def test_two_rank_combine_matches_oracle(rho, T):
    """Criterion fires within T lags (fast-mixing chains): identical to the reference."""
    q = _ar1(6, 81, 5, rho, seed=11)                                   # 40 samples per half
    out = _run(q, T)
    R_ref, neff_ref = O.convergence_stats(q, thin_rate=1, warm_up_num=0)
    for rank in (0, 1):
        R, neff = out[rank]
        np.testing.assert_allclose(R, R_ref, rtol=1e-12)
        np.testing.assert_allclose(neff, neff_ref, rtol=1e-12)


def test_two_rank_all_lags_matches_oracle_slow_mixing():
    """Slowly mixing chains with every lag available (T >= n - 1): identical to the reference."""
    q = _ar1(4, 33, 3, 0.9, seed=5)                                    # n = 16
    out = _run(q, 16)                                                  # T = 16 >= n - 1
    R_ref, neff_ref = O.convergence_stats(q, thin_rate=1, warm_up_num=0)
    R, neff = out[0]
    np.testing.assert_allclose(R, R_ref, rtol=1e-12)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-12)


def test_single_rank_equals_two_ranks():
    q = _ar1(8, 65, 4, 0.5, seed=3)
    two = _run(q, 32)
    one = _run(q, 32, world=1)
    np.testing.assert_allclose(two[0][0], one[0][0], rtol=1e-13)
    np.testing.assert_allclose(two[0][1], one[0][1], rtol=1e-13)
