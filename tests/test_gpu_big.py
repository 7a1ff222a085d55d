"""Targets beyond the fused kernels' register budget (hmc_big.hip): dense precision with D > 128
and diagonal precision with D > 2048 (the reference's dgemv takes any D, samplers.py:835-837).

Replay mode vs the oracle (oracle/hmc_oracle.py restating samplers.py:387-491) on the same draws:
identical accept counts and leapfrog totals, q_chain within 1e-9, E within 1e-10 relative (MFMA
k-ordered sums vs BLAS).  Philox mode: determinism and the stationary law at a few thousand chains."""
import numpy as np
import pytest
import torch

from oracle import hmc_oracle as O

pytestmark = pytest.mark.gpu


class FastMVN(O.MVNTarget):
    """V = 0.5 (logdet const + x.P.x) instead of scipy's eigh-based logpdf (same value to ~1e-14)."""

    def __init__(self, q0, cov0):
        super().__init__(q0, cov0)
        D = self.q0.size
        self.c = D * np.log(2 * np.pi) + np.linalg.slogdet(self.cov0)[1]

    def V(self, q):
        x = q - self.q0
        return 0.5 * (self.c + x @ (self.inv_cov0 @ x))


def _replay(D, cov, q0, dt, fp_mode, N=3, Niter=10, wu=3, thin=1, L=(3, 9), cov_p=None):
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    rs = np.random.RandomState(D)
    q_start = q0 + rs.standard_normal((N, D))
    full = cov_p is not None and np.any(cov_p - np.diag(np.diag(cov_p)))
    if full:                                      # momenta ~ N(0, cov_p) as the reference draws them
        C = np.linalg.cholesky(cov_p)
        p0 = rs.standard_normal((N, D)) @ C.T
        P = rs.standard_normal((N, Niter, D)) @ C.T
    else:
        scale = np.sqrt(np.diag(cov_p)) if cov_p is not None else np.ones(D)
        p0 = rs.standard_normal((N, D)) * scale
        P = rs.standard_normal((N, Niter, D)) * scale
    Ls = rs.randint(L[0], L[1], size=(N, Niter)).astype(np.int32)
    lnu = np.log(rs.random_sample((N, Niter)))
    tgt = FastMVN(q0, cov)
    ref = O.gen_sample_random(O.HMCCore(tgt, dt, cov_p), q_start, N, Niter, wu, thin, L[0], L[1],
                              O.ReplayDraws(p0, P, Ls, lnu))
    from hmc_amd.engine import RandomEngine
    eng = RandomEngine(MVNTarget(q0, cov, logdet_const=tgt.c), N, Niter, wu, thin, L[0], L[1], dt, cov_p=cov_p,
                       rng="replay", fp_mode=fp_mode)
    assert eng._order is not None            # the large-D workspace
    eng.set_replay(p0, P, Ls, lnu)
    eng.init(q_start)
    eng.run(1, 5)
    eng.run(5, Niter + 1)
    torch.cuda.synchronize()
    return eng, ref, Ls


def _check(eng, ref, Ls):
    from hmc_amd import _lib as H
    c = eng.read_counters()
    assert int(c[H.CNT_ACCEPT]) == ref["accept_count"]
    assert int(c[H.CNT_ACCEPT_WU]) == ref["accept_count_warm_up"]
    assert int(c[H.CNT_LEAPFROG]) == int(Ls.sum())
    np.testing.assert_allclose(eng.q_chain.cpu().numpy(), ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.E_chain.cpu().numpy(), ref["E_chain"], rtol=1e-10)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
@pytest.mark.parametrize("D,rho", [(136, 0.9), (300, 0.5)])
def test_dense_large_D_vs_oracle(D, rho, fp_mode):
    q0 = np.linspace(-0.5, 0.5, D)
    eng, ref, Ls = _replay(D, O.mvn_cov(D, rho), q0, 0.05, fp_mode)
    _check(eng, ref, Ls)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
@pytest.mark.parametrize("D", [136, 300])
def test_dense_large_D_full_cov_p_vs_oracle(D, fp_mode):
    """A full (non-diagonal) cov_p above D = 128 (samplers.py:352-356: p ~ N(0, cov_p),
    K = p.inv(cov_p).p/2, kick by inv(cov_p).dVdq, :811-839): the large-D path's extra GEMMs
    (kick = inv_cov_p . g, inv_cov_p p at both energies) vs the oracle on the same draws."""
    import make_golden_shapes as S
    eng, ref, Ls = _replay(D, O.mvn_cov(D, 0.7), np.linspace(-0.3, 0.3, D), 0.05, fp_mode, cov_p=S.dense_cov_p(D))
    _check(eng, ref, Ls)
    np.testing.assert_allclose(eng.dE_chain.cpu().numpy(), ref["dE_chain"], rtol=1e-8, atol=1e-9)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_diagonal_large_D_vs_oracle(fp_mode):
    D = 2050
    rs = np.random.RandomState(1)
    cov = np.diag(rs.uniform(0.5, 2.0, D))
    dt = rs.uniform(0.05, 0.1, D)
    cov_p = np.diag(rs.uniform(0.8, 1.25, D))
    eng, ref, Ls = _replay(D, cov, np.zeros(D), dt, fp_mode, N=2, Niter=6, wu=1, thin=2, cov_p=cov_p)
    _check(eng, ref, Ls)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
@pytest.mark.parametrize("D,dense", [(136, True), (2050, False)])
def test_large_D_chain0_capture_vs_oracle(D, dense, fp_mode):
    """Chain-0 trajectory capture above the fused kernels' limits (samplers.py:442-475, make_movie's
    input): phi_q (q[:2] at the start and after every leapfrog step of the first N_save iterations)
    and decision_chain from the large-D path equal the oracle's on the same replayed draws
    (this returned HMC_ENOTSUP)."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, Niter, wu, n_save, dt = 3, 12, 2, 7, 0.08
    rs = np.random.RandomState(D + 5)
    cov = O.mvn_cov(D, 0.6) if dense else np.diag(rs.uniform(0.5, 2.0, D))
    tgt = FastMVN(np.zeros(D), cov)
    q_start = rs.standard_normal((N, D))
    p0, P = rs.standard_normal((N, D)), rs.standard_normal((N, Niter, D))
    Ls = rs.randint(3, 9, size=(N, Niter)).astype(np.int32)
    lnu = np.log(rs.random_sample((N, Niter)))
    eng = RandomEngine(MVNTarget(np.zeros(D), cov, logdet_const=tgt.c), N, Niter, wu, 1, 3, 9, dt, rng="replay",
                       fp_mode=fp_mode, n_save=n_save)
    eng.set_replay(p0, P, Ls, lnu)
    eng.init(q_start)
    eng.run(1, 6)
    eng.run(6, Niter + 1)
    ref = O.gen_sample_random(O.HMCCore(tgt, dt), q_start, N, Niter, wu, 1, 3, 9, O.ReplayDraws(p0, P, Ls, lnu),
                              n_save_chain0=n_save)
    traj, tl = eng.traj.cpu().numpy(), eng.traj_len.cpu().numpy()
    np.testing.assert_array_equal(eng.decision.cpu().numpy(), ref["decision_chain"][:n_save])
    assert len(ref["phi_q"]) == n_save
    for i, want in enumerate(ref["phi_q"]):
        assert tl[i] == want.shape[0] == Ls[0, i] + 1
        np.testing.assert_allclose(traj[i, :tl[i]], want, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.q_chain.cpu().numpy(), ref["q_chain"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("D,rho,dense,full_p", [(160, 0.8, True, False), (2100, 0.0, False, False),
                                               (160, 0.8, True, True)])
def test_large_D_philox_stationary(D, rho, dense, full_p):
    """Chains started in N(0, Sigma) stay there (per-dim variance 1, corr rho), also with a full
    cov_p (Philox momenta p = C z); runs repeat.  With a cov_p other than the identity the
    reference's leapfrog (Q3: kick by inv(cov_p).dVdq, drift by p, samplers.py:831-839) does not
    conserve p.inv(cov_p).p/2 + V: the map is still a volume-preserving, reversible shear pair, so
    the law is right, but acceptance is low (0 of 1024 at dt = 0.1 for this cov_p, diagonal or
    not, against 983 with cov_p = I): that case runs at dt = 0.02."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    import make_golden_shapes as S
    cov = O.mvn_cov(D, rho) if dense else np.eye(D)
    N = 2048
    qs = np.random.RandomState(3).standard_normal((N, D)) @ np.linalg.cholesky(cov).T

    def run():
        h = HMC_sampler(D, None, None, Nchain=N, Niter=4, sampler_type="Random", L_low=5, L_high=12,
                        dt=0.02 if full_p else 0.1,
                        warm_up_num=1, target=MVNTarget(np.zeros(D), cov), rng="philox", seed=8, fp_mode="fast",
                        cov_p=S.dense_cov_p(D) if full_p else None)
        h.gen_sample(qs, verbose=False)
        return h
    h = run()
    last = h.q_chain[:, -1, :]
    assert np.abs(last.var(axis=0).mean() - 1) < 6 * np.sqrt(2 / (N * D)) + 0.01
    if dense:
        assert abs(np.corrcoef(last[:, 0], last[:, 1])[0, 1] - rho) < 6 * (1 - rho ** 2) / np.sqrt(N) + 0.01
    assert (0.05 if full_p else 0.3) < h.accept_R <= 1.0
    assert np.array_equal(h.q_chain, run().q_chain)
