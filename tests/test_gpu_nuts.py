"""NUTS on the GPU (hmc_nuts_iters) against the reference fixture and the oracle.

The reference consumes its NUTS draws from the global np.random in a data-dependent order
(directions :608, progressive-sampling uniforms :750, sub-tree uniforms :773), so parity runs
replay an explicit per-chain tape: the recorded one for the reference fixture
(tests/golden/f6_nuts_dense100.npz, made by tests/golden/make_golden.py), synthetic ones for
the oracle cases.  Decisions (U-turns, instability, uniform comparisons) must agree exactly;
states agree to round-off (MFMA k-ordered gradient sums vs BLAS): q_chain 1e-9, E 1e-10 rel.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import hmc_oracle as O

pytestmark = pytest.mark.gpu


def _nuts(D, tgt, Nchain, Niter, wu, thin, dt, d_max, cov_p=None, **kw):
    from hmc_amd.samplers import HMC_sampler
    return HMC_sampler(D, None, None, Nchain=Nchain, Niter=Niter, thin_rate=thin, warm_up_num=wu,
                       sampler_type="NUTS", dt=dt, d_max=d_max, cov_p=cov_p, target=tgt, **kw)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_nuts_replay_matches_reference(fp_mode):
    from hmc_amd.target import MVNTarget
    g = load_golden("f6_nuts_dense100.npz")
    m = g["meta"]
    h = _nuts(m["D"], MVNTarget(g["q0"], g["cov0"]), m["Nchain"], m["Niter"], m["warm_up"], m["thin"],
              m["dt"], m["d_max"], rng="replay", fp_mode=fp_mode)
    h.set_nuts_replay(g["p0"], g["p"], g["tape"])
    h.gen_sample(g["q_start"], verbose=False)
    assert h.n_leapfrog == int(g["n_leapfrog"])
    assert h.N_total_steps == int(g["N_total_steps"])
    assert h.accept_R == 1.0 and h.accept_R_warm_up == 1.0
    np.testing.assert_allclose(h.q_chain, g["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], g["E_chain"], rtol=1e-10)
    np.testing.assert_allclose(h.dE_chain[:, :, 0], g["dE_chain"], rtol=1e-8, atol=1e-9)
    h.compute_convergence_stats()
    np.testing.assert_allclose(h.R_q, g["R_q"], rtol=1e-6)


CASES = [
    # D, rho, q0 scale, Nchain, Niter, wu, thin, dt, d_max, cov_p diag?, dt vector?, on_dmax
    (5, 0.0, 0.0, 6, 15, 3, 1, 0.2, 8, False, False, "raise"),
    (37, 0.5, 1.0, 5, 12, 0, 2, 0.15, 9, True, False, "break"),        # d_max reached, mass matrix
    (16, 0.9, 0.0, 4, 10, 2, 3, 0.1, 10, False, True, "raise"),
    (100, 0.95, 0.5, 3, 4, 1, 1, 0.1, 12, False, False, "raise"),
    (10, 0.99, 0.0, 4, 8, 0, 1, 0.9, 8, False, False, "raise"),       # large dt: |E-E0| > 1000 guard
    (8, 0.3, 0.0, 5, 10, 2, 1, 0.05, 3, False, False, "break"),       # d_max reached
    (128, 0.7, 0.0, 2, 4, 0, 1, 0.1, 11, False, False, "raise"),
    (1, 0.0, 0.0, 3, 20, 5, 1, 0.3, 8, False, False, "raise"),
]


@pytest.mark.parametrize("case", CASES, ids=[f"D{c[0]}_rho{c[1]}_dt{c[7]}_dmax{c[8]}" for c in CASES])
@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_nuts_matches_oracle(case, fp_mode):
    from hmc_amd.target import MVNTarget
    D, rho, qs, N, Niter, wu, thin, dt, d_max, diag_p, dtvec, on_dmax = case
    rs = np.random.RandomState(1000 + D)
    cov = O.mvn_cov(D, rho) if rho > 0 else np.eye(D)
    q0 = rs.standard_normal(D) * qs
    cov_p = np.diag(rs.uniform(0.5, 2.0, D)) if diag_p else None
    dts = rs.uniform(0.5, 1.0, D) * dt if dtvec else dt
    q_start = q0 + rs.standard_normal((N, D)) * 1.5
    scale = np.sqrt(np.diag(cov_p)) if diag_p else np.ones(D)
    p0 = rs.standard_normal((N, D)) * scale
    P = rs.standard_normal((N, Niter, D)) * scale
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))   # int(v) = direction, v = uniform
    core = O.HMCCore(O.MVNTarget(q0, cov), dts, cov_p)
    ref = O.gen_sample_nuts(core, q_start, N, Niter, wu, thin, d_max, O.ReplayDraws(p0, P, tape=tape.copy()),
                            on_dmax=on_dmax)
    h = _nuts(D, MVNTarget(q0, cov), N, Niter, wu, thin, dts, d_max, cov_p=cov_p, rng="replay", fp_mode=fp_mode)
    h.set_nuts_replay(p0, P, tape)
    h.gen_sample_NUTS(q_start, 0, False, on_dmax=on_dmax)
    assert h.n_leapfrog == ref["n_leapfrog"]
    assert h.n_unstable == ref["n_unstable"]
    assert h.N_total_steps == ref["N_total_steps"]
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(h.dE_chain[:, :, 0], ref["dE_chain"], rtol=1e-8, atol=1e-9)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_nuts_deep_tree_single_chain_handoff(fp_mode):
    """One chain, d_max = 14 and a step small enough for 2^12 .. 2^13-point trees (unit MVN, D = 2,
    dt = 2e-3: 16,381 leapfrogs over 3 iterations), every iteration in ONE launch.  Iterations
    2 and 3 are queued units of the same chain, so their slots wait thousands of wave steps for
    the hand-off of the one before (samplers.py:595-598 with the deepest trees this d_max allows
    short of the abort): no give-up may trip, and leapfrog counts and q_chain equal the oracle's."""
    from hmc_amd.target import MVNTarget
    D, N, Niter, d_max, dt = 2, 1, 3, 14, 2e-3
    rs = np.random.RandomState(3)
    q_start = rs.standard_normal((N, D))
    p0 = rs.standard_normal((N, D))
    P = rs.standard_normal((N, Niter, D))
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))
    core = O.HMCCore(O.MVNTarget(np.zeros(D), np.eye(D)), dt, None)
    ref = O.gen_sample_nuts(core, q_start, N, Niter, 0, 1, d_max, O.ReplayDraws(p0, P, tape=tape.copy()),
                            on_dmax="raise")
    assert ref["n_leapfrog"] == 16381
    h = _nuts(D, MVNTarget(np.zeros(D), np.eye(D)), N, Niter, 0, 1, dt, d_max, rng="replay", fp_mode=fp_mode)
    h.set_nuts_replay(p0, P, tape)
    h.gen_sample_NUTS(q_start, 0, False)              # raises on a give-up (CNT_HANDOFF_GIVEUP)
    from hmc_amd import _lib as H
    c = h.engine.read_counters()
    assert c[H.CNT_HANDOFF_GIVEUP] == 0 and c[H.CNT_DMAX] == 0
    assert h.n_leapfrog == ref["n_leapfrog"]
    assert h.N_total_steps == ref["N_total_steps"]
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-10, atol=1e-10)


def test_nuts_d_max_beyond_15_deep_tree():
    """d_max above the former bound of 15 (the reference takes any d_max, samplers.py:306,
    :519-520): one chain, D = 2, dt small enough that a tree needs more than 2^15 points before both
    ends turn.  Leapfrog counts, q_chain and E equal the oracle's on the same
    replayed draws, with no d_max hit and no hand-off give-up."""
    from hmc_amd import _lib as H
    from hmc_amd.target import MVNTarget
    D, N, Niter, d_max, dt = 2, 1, 2, 20, 1.2e-4
    rs = np.random.RandomState(5)
    q_start = rs.standard_normal((N, D))
    p0 = rs.standard_normal((N, D))
    P = rs.standard_normal((N, Niter, D))
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * ((1 << 17) + d_max + 2)))
    core = O.HMCCore(O.MVNTarget(np.zeros(D), np.eye(D)), dt, None)
    ref = O.gen_sample_nuts(core, q_start, N, Niter, 0, 1, d_max, O.ReplayDraws(p0, P, tape=tape.copy()),
                            on_dmax="raise")
    assert ref["n_leapfrog"] > 1 << 16                 # trees deeper than 15 doublings
    h = _nuts(D, MVNTarget(np.zeros(D), np.eye(D)), N, Niter, 0, 1, dt, d_max, rng="replay", fp_mode="exact")
    h.set_nuts_replay(p0, P, tape)
    h.gen_sample_NUTS(q_start, 0, False)
    c = h.engine.read_counters()
    assert c[H.CNT_HANDOFF_GIVEUP] == 0 and c[H.CNT_DMAX] == 0
    assert h.n_leapfrog == ref["n_leapfrog"]
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-10, atol=1e-10)


def test_nuts_replay_without_tape_warns():
    """rng='replay' NUTS without set_nuts_replay cannot follow the reference's data-dependent
    np.random order (samplers.py:608, :748, :773): it runs Philox seeded from np.random and says so."""
    from hmc_amd.target import MVNTarget
    D, N = 3, 4
    h = _nuts(D, MVNTarget(np.zeros(D), np.eye(D)), N, 3, 0, 1, 0.2, 6, rng="replay")
    np.random.seed(1)
    with pytest.warns(UserWarning, match="Philox"):
        h.gen_sample(np.zeros((N, D)), verbose=False)
    np.random.seed(1)
    h2 = _nuts(D, MVNTarget(np.zeros(D), np.eye(D)), N, 3, 0, 1, 0.2, 6, rng="replay")
    with pytest.warns(UserWarning):
        h2.gen_sample(np.zeros((N, D)), verbose=False)
    assert np.array_equal(h.q_chain, h2.q_chain)     # np.random.seed still fixes the run


def test_nuts_dmax_raises():
    from hmc_amd.target import MVNTarget
    D = 4
    h = _nuts(D, MVNTarget(np.zeros(D), np.eye(D)), 8, 3, 0, 1, 0.01, 1, rng="philox", seed=1)
    with pytest.raises(AssertionError):
        h.gen_sample(np.ones((8, D)), verbose=False)


def test_nuts_tape_exhaustion_raises():
    from hmc_amd.target import MVNTarget
    D, N = 3, 2
    h = _nuts(D, MVNTarget(np.zeros(D), np.eye(D)), N, 4, 0, 1, 0.1, 6, rng="replay")
    h.set_nuts_replay(np.ones((N, D)), np.ones((N, 4, D)), np.full((N, 2), 0.5))
    with pytest.raises(IndexError):
        h.gen_sample(np.zeros((N, D)), verbose=False)


@pytest.mark.parametrize("D,rho", [(100, 0.95), (24, 0.5)])
def test_nuts_philox_statistics(D, rho):
    """Philox streams at scale, chains started in the stationary law N(0, Sigma): NUTS leaves
    it invariant, so per-dim variances stay 1 and corr(q0, q1) = rho; runs are deterministic."""
    from hmc_amd.target import MVNTarget
    cov = O.mvn_cov(D, rho)
    N = 4096
    qs = np.random.RandomState(D).standard_normal((N, D)) @ np.linalg.cholesky(cov).T

    def run():
        h = _nuts(D, MVNTarget(np.zeros(D), cov), N, 6, 1, 1, 0.1, 12, rng="philox", seed=5, fp_mode="fast",
                  iters_per_launch=3)
        h.gen_sample(qs, verbose=False)
        return h
    h = run()
    last = h.q_chain[:, -1, :]
    assert np.abs(last.var(axis=0) - 1).max() < 6 * np.sqrt(2 / N)
    assert abs(np.corrcoef(last[:, 0], last[:, 1])[0, 1] - rho) < 6 * (1 - rho ** 2) / np.sqrt(N) + 0.01
    assert h.n_leapfrog > N * 6 * 3
    h2 = run()
    assert np.array_equal(h.q_chain, h2.q_chain)


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_nuts_full_cov_p_matches_oracle(fp_mode):
    """NUTS with a full (non-diagonal) cov_p (Q3: p ~ N(0, cov_p), K = p.inv(cov_p).p/2, kick by
    inv(cov_p).dVdq; samplers.py:352-356, :811-839 through gen_sample_NUTS :495-808), replayed
    draws vs the oracle; plus Philox determinism."""
    from hmc_amd.target import MVNTarget
    import make_golden_shapes as S
    D, N, Niter, wu, dt, d_max = 12, 5, 10, 2, 0.15, 9
    rs = np.random.RandomState(77)
    cov, cov_p = O.mvn_cov(D, 0.6), S.dense_cov_p(D)
    C = np.linalg.cholesky(cov_p)
    q_start = rs.standard_normal((N, D)) * 1.5
    p0 = rs.standard_normal((N, D)) @ C.T
    P = rs.standard_normal((N, Niter, D)) @ C.T
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))
    core = O.HMCCore(O.MVNTarget(np.zeros(D), cov), dt, cov_p)
    ref = O.gen_sample_nuts(core, q_start, N, Niter, wu, 1, d_max, O.ReplayDraws(p0, P, tape=tape.copy()),
                            on_dmax="break")
    h = _nuts(D, MVNTarget(np.zeros(D), cov), N, Niter, wu, 1, dt, d_max, cov_p=cov_p, rng="replay",
              fp_mode=fp_mode)
    h.set_nuts_replay(p0, P, tape)
    h.gen_sample_NUTS(q_start, 0, False, on_dmax="break")
    assert h.n_leapfrog == ref["n_leapfrog"]
    assert h.N_total_steps == ref["N_total_steps"]
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-10, atol=1e-10)
    runs = []
    for _ in range(2):
        g = _nuts(D, MVNTarget(np.zeros(D), cov), 64, 6, 1, 1, dt, d_max, cov_p=cov_p, rng="philox", seed=3,
                  fp_mode=fp_mode)
        g.gen_sample_NUTS(q_start[np.arange(64) % N], 0, False, on_dmax="break")
        runs.append(g.q_chain)
    assert np.array_equal(runs[0], runs[1]) and np.isfinite(runs[0]).all()
