"""Edge cases of the GPU samplers against the oracle (replayed draws, bit-exact in exact mode):
empty and ragged chain counts, the kernel-selection boundaries (lane groups up to D = 64, one
wave per chain from D = 65, the largest diagonal D = 2048), constant trajectory length, and the
shapes the kernels refuse (reference: NotImplementedError-style HMC_ENOTSUP)."""
import numpy as np
import pytest
import torch

from oracle import hmc_oracle as O

pytestmark = pytest.mark.gpu


def _replay_vs_oracle(D, N, Niter=12, wu=3, thin=1, lo=3, hi=9, seed=0):
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    rs = np.random.RandomState(seed + D)
    q0, cov0 = np.zeros(D), np.eye(D)
    tgt = O.MVNTarget(q0, cov0)
    h = HMC_sampler(D, tgt.V, tgt.dVdq, Nchain=N, Niter=Niter, sampler_type="Random", L_low=lo, L_high=hi, dt=0.1,
                    thin_rate=thin, warm_up_num=wu, target=MVNTarget(q0, cov0))
    q_start = rs.standard_normal((N, D))
    np.random.seed(seed)
    h.gen_sample(q_start, verbose=False)
    np.random.seed(seed)
    ref = O.gen_sample_random(O.HMCCore(tgt, 0.1), q_start, N, Niter, wu, thin, lo, hi, O.LiveDraws(D, h.cov_p))
    assert np.array_equal(h.q_chain, ref["q_chain"])
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-12)
    assert h.accept_R == ref["accept_R"]
    assert h.N_total_steps == ref["N_total_steps"]
    return h


@pytest.mark.parametrize("D", [1, 3, 64, 65, 127, 129])
def test_kernel_boundaries_bitexact(D):
    """D = 1, 3 (odd, lane groups), 64 / 65 (last lane-group shape / first wave-per-chain shape),
    127 / 129 (K = 1 / K = 2 of the wave kernel)."""
    _replay_vs_oracle(D, N=5)


@pytest.mark.parametrize("N", [1, 5, 17, 67])
def test_ragged_chain_counts_bitexact(N):
    """Chain counts that leave partial waves / lane groups / 4-wave blocks."""
    _replay_vs_oracle(100, N=N, Niter=8)
    _replay_vs_oracle(10, N=N, Niter=8)


def test_largest_diagonal_dimension_bitexact():
    """D = 2048: 16 coordinate pairs per lane, the widest wave-kernel instance (one chain, two
    iterations: the oracle's eigh/SVD per energy and draw take ~10 s at this size)."""
    _replay_vs_oracle(2048, N=1, Niter=2, wu=0)


def test_constant_trajectory_length():
    """L_high = L_low + 1: randint returns L_low every time (Q1)."""
    h = _replay_vs_oracle(100, N=4, lo=7, hi=8)
    assert h.n_leapfrog == 4 * h.Niter * 7


def test_empty_chain_batch():
    """Nchain = 0 through the engine: nothing launched, nothing counted."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    for cov in (np.eye(100), O.mvn_cov(100, 0.5)):
        eng = RandomEngine(MVNTarget(np.zeros(100), cov), 0, 10, 2, 1, 5, 20, 0.1, rng="philox")
        eng.init(np.zeros((0, 100)))
        eng.run(1, 11)
        torch.cuda.synchronize()
        assert eng.q_chain.shape == (0, eng.L_chain, 100)
        assert int(eng.read_counters().sum()) == 0


def test_unsupported_shapes_raise():
    """What the kernels still leave out raises NotImplementedError with no launch: d_max beyond 30
    (2^30 - 1 leapfrogs per tree; the reference takes any d_max).  Chain-0 trajectory
    capture above D = 128, refused up to round 4, runs now (tests/test_gpu_big.py)."""
    from hmc_amd.engine import NutsEngine
    from hmc_amd.target import MVNTarget
    with pytest.raises(NotImplementedError):
        NutsEngine(MVNTarget(np.zeros(8), np.eye(8)), 2, 4, 0, 1, 31, 0.1, rng="philox")
    NutsEngine(MVNTarget(np.zeros(8), np.eye(8)), 2, 4, 0, 1, 30, 0.1, rng="philox")   # the bound itself
