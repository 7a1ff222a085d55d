"""GPU parity of the Random-trajectory engine (hmc_random_iters) against the reference.

Replay mode feeds the kernels the exact draws the reference consumed (golden
fixtures recorded from the reference itself, tests/golden/make_golden.py), so:
  * diagonal targets, fp_mode="exact": q_chain BIT-EXACT, acceptance counts,
    N_total_steps and the chain-0 trajectory capture exact; E_chain within 1e-12
    relative (energy sums are re-associated vs scipy's eigh-based logpdf);
  * fp_mode="fast" (FMA-contracted integrator): q_chain within 1e-9 relative,
    identical accept decisions on these fixtures.
Philox mode at BASELINE sizes is checked through size-independent properties
(determinism, shard invariance, moments, acceptance).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import hmc_oracle as O

pytestmark = pytest.mark.gpu

DIAG_FIXTURES = ["f1_case1a.npz", "f2_case1c_small.npz", "f8_diag_thin_vecdt.npz", "f9_wu0_thin2.npz",
                 "f10_case2a.npz"]


def _sampler_from_golden(g, **kw):
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    m = g["meta"]
    dt = g["dt"]
    dt = float(dt) if dt.ndim == 0 else dt
    tgt = O.MVNTarget(g["q0"], g["cov0"])
    # explicit target: exact q0 / inv(cov0) as the reference computed them (probing is exact only for q0 = 0)
    return HMC_sampler(m["D"], tgt.V, tgt.dVdq, Nchain=m["Nchain"], Niter=m["Niter"], sampler_type="Random",
                       L_low=m["L_low"], L_high=m["L_high"], dt=dt, thin_rate=m["thin"], warm_up_num=m["warm_up"],
                       cov_p=g["cov_p"], target=MVNTarget(g["q0"], g["cov0"]), **kw)


def _run_replay(g, fp_mode="exact"):
    """Run the product in replay mode on the recorded streams: the live global RNG is
    re-seeded and re-advanced past start_pts exactly as in the reference run."""
    m = g["meta"]
    h = _sampler_from_golden(g, fp_mode=fp_mode)
    np.random.seed(m["seed"])
    np.random.multivariate_normal(np.zeros(m["D"]), np.diag(np.ones(m["D"])) * m["start_scale"], size=m["Nchain"])
    h.gen_sample(g["q_start"], N_save_chain0=m["n_save"], verbose=False)
    return h


@pytest.mark.parametrize("fx", DIAG_FIXTURES)
def test_replay_exact_matches_reference(fx):
    g = load_golden(fx)
    m = g["meta"]
    h = _run_replay(g, "exact")
    assert np.array_equal(h.q_chain, g["q_chain"]), "q_chain not bit-identical to the reference"
    np.testing.assert_allclose(h.E_chain[:, :, 0], g["E_chain"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(h.dE_chain[:, :, 0], g["dE_chain"], rtol=1e-9, atol=1e-11)
    assert h.accept_R == float(g["accept_R"])
    if m["warm_up"] > 0:
        assert h.accept_R_warm_up == float(g["accept_R_warm_up"])
    assert h.N_total_steps == int(g["N_total_steps"])
    assert h.n_leapfrog == int(g["n_leapfrog"])
    if m["n_save"]:
        assert np.array_equal(h.decision_chain[:, 0], g["decision_chain"])
        assert np.array_equal(np.concatenate(h.phi_q), g["phi_q_flat"])


@pytest.mark.parametrize("fx", DIAG_FIXTURES)
def test_replay_fast_within_tolerance(fx):
    g = load_golden(fx)
    h = _run_replay(g, "fast")
    np.testing.assert_allclose(h.q_chain, g["q_chain"], rtol=1e-9, atol=1e-9)
    assert h.accept_R == float(g["accept_R"])


@pytest.mark.parametrize("fx", ["f1_case1a.npz", "f2_case1c_small.npz", "f9_wu0_thin2.npz"])
def test_convergence_stats_on_device(fx):
    """R-hat / ESS / per-dim mean,std computed by the diagnostics kernels vs the reference
    values (north_star tolerance 1e-6 rel; observed ~1e-13)."""
    g = load_golden(fx)
    h = _run_replay(g, "exact")
    h.compute_convergence_stats()
    np.testing.assert_allclose(h.R_q, g["R_q"], rtol=1e-10)
    np.testing.assert_allclose(h.n_eff_q, g["n_eff_q"], rtol=1e-8)
    from hmc_amd.diagnostics import per_dim_mean_std
    mean, std = per_dim_mean_std(h.q_chain_device)
    np.testing.assert_allclose(mean, g["mean"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(std, g["std"], rtol=1e-10)


def test_convergence_stats_vectors_device():
    """utils.convergence_stats on the reference's synthetic AR(1) vectors (incl. thinning,
    warm-up offsets, odd lengths)."""
    from hmc_amd.diagnostics import convergence_stats
    g = load_golden("f5_convergence.npz")
    for tag in "abcdf":
        x = g[f"{tag}_x"]
        R, neff = convergence_stats(x, warm_up_num=0, thin_rate=1)
        np.testing.assert_allclose(R, g[f"{tag}_R"], rtol=1e-10)
        np.testing.assert_allclose(neff, g[f"{tag}_neff"], rtol=1e-8)
        R5, neff5 = convergence_stats(x, thin_rate=5, warm_up_num=3)
        np.testing.assert_allclose(R5, g[f"{tag}_R_thin5"], rtol=1e-10)
        np.testing.assert_allclose(neff5, g[f"{tag}_neff_thin5"], rtol=1e-8)


@pytest.mark.parametrize("thin,wu", [(1, 0), (3, 7)])
def test_convergence_stats_long_lags_vs_oracle(thin, wu):
    """Slowly mixing AR(1) chains (rho up to 0.997, mean 3): the reference's ESS loop reads lags far
    past the first pass's 96, so the undecided dims read every remaining lag in ONE more pass (the
    window is read at most twice); R-hat and ESS still equal the oracle's convergence_stats
    (utils.py:77-179 restated)."""
    from hmc_amd import diagnostics as G
    rs = np.random.RandomState(3)
    # split halves of n = 300 (thin 1) and 299 (thin 3): past the complete pass (n - 1 <= 256)
    N, L, D, rho = 20, 601 if thin == 1 else 1801, 12, np.linspace(0.3, 0.997, 12)
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D)) + 3.0
    for t in range(1, L):
        x[:, t] = 3.0 + rho * (x[:, t - 1] - 3.0) + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    R, neff = G.convergence_stats(x, thin_rate=thin, warm_up_num=wu)
    assert G.LAST_INFO["fallback_dims"] > 0 and G.LAST_INFO["lags"] > 96
    assert G.LAST_INFO["fallback_passes"] == 1
    R_ref, neff_ref = O.convergence_stats(x, thin_rate=thin, warm_up_num=wu)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)


def test_leapfrog_and_energy_vectors():
    """Batched leap_frog / E (samplers.py:811-839) vs the reference's single-call outputs."""
    g = load_golden("f4_leapfrog.npz")
    for tag, exact in (("unit100", True), ("diag10_vecdt", True), ("dense100", False)):
        from hmc_amd.samplers import HMC_sampler
        tgt = O.MVNTarget(g[f"{tag}_q0"], g[f"{tag}_cov0"])
        dt = g[f"{tag}_dt"]
        from hmc_amd.target import MVNTarget
        h = HMC_sampler(tgt.q0.size, tgt.V, tgt.dVdq, Nchain=2, Niter=1, sampler_type="Random", L_low=1,
                        L_high=2, dt=float(dt) if dt.ndim == 0 else dt, cov_p=g[f"{tag}_cov_p"],
                        target=MVNTarget(g[f"{tag}_q0"], g[f"{tag}_cov0"]))
        pn, qn = h.leap_frog(g[f"{tag}_p"], g[f"{tag}_q"])
        if exact:
            assert np.array_equal(pn, g[f"{tag}_pn"]) and np.array_equal(qn, g[f"{tag}_qn"])
        else:  # dense BLAS dgemv summation order is unspecified
            np.testing.assert_allclose(pn, g[f"{tag}_pn"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(qn, g[f"{tag}_qn"], rtol=1e-13, atol=1e-13)
        E = h.E(g[f"{tag}_q"], g[f"{tag}_p"])
        np.testing.assert_allclose(E, g[f"{tag}_E"], rtol=1e-12)


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors."""
    from hmc_amd import _lib as H
    L = H.lib()
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    kats = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
            ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
            ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
             (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kats:
        H.check(L.hmc_philox(*ctr, *key, 1, out.data_ptr(), None))
        got = tuple(int(v) & 0xffffffff for v in out.cpu().numpy())
        assert got == want


def test_philox_normals_moments():
    from hmc_amd import _lib as H
    L = H.lib()
    n, npairs = 1 << 16, 8
    out = torch.empty((n, 2 * npairs), dtype=torch.float64, device="cuda")
    H.check(L.hmc_rng_normals(7, 0, n, 3, npairs, out.data_ptr(), None))
    z = out.cpu().numpy().ravel()
    N = z.size
    assert abs(z.mean()) < 5 / np.sqrt(N)
    assert abs(z.var() - 1) < 5 * np.sqrt(2 / N)
    assert abs(np.mean(z ** 3)) < 5 * np.sqrt(15 / N)
    assert abs(np.mean(z ** 4) - 3) < 5 * np.sqrt(96 / N)
    # independent streams: correlation between the two normals of a pair and across chains
    assert abs(np.corrcoef(out[:, 0].cpu(), out[:, 1].cpu())[0, 1]) < 5 / np.sqrt(n)
    assert abs(np.corrcoef(out[:-1, 0].cpu(), out[1:, 0].cpu())[0, 1]) < 5 / np.sqrt(n)


def _philox_run(N, D, Niter, wu, seed=1, offset=0, fp_mode="fast", target=None, ipl=None):
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    t = target or MVNTarget(np.zeros(D), np.eye(D))
    h = HMC_sampler(D, None, None, Nchain=N, Niter=Niter, sampler_type="Random", L_low=5, L_high=20, dt=0.1,
                    warm_up_num=wu, target=t, rng="philox", seed=seed, fp_mode=fp_mode, chain_offset=offset,
                    iters_per_launch=ipl)
    rs = np.random.RandomState(seed + 1000 + offset)
    q0 = rs.standard_normal((N, D)) * np.sqrt(2)
    h.gen_sample(q0, verbose=False)
    return h, q0


def test_philox_deterministic_and_shard_invariant():
    """Results are a pure function of (seed, global chain id): identical across runs, launch
    splits (iters_per_launch) and chain shards (chain_offset), as multi-GPU sharding needs."""
    N, D = 4096, 100
    h1, q0 = _philox_run(N, D, 12, 4)
    h2, _ = _philox_run(N, D, 12, 4, ipl=5)
    assert np.array_equal(h1.q_chain, h2.q_chain)
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    half = N // 2
    parts = []
    for off in (0, half):
        h = HMC_sampler(D, None, None, Nchain=half, Niter=12, sampler_type="Random", L_low=5, L_high=20, dt=0.1,
                        warm_up_num=4, target=MVNTarget(np.zeros(D), np.eye(D)), rng="philox", seed=1,
                        fp_mode="fast", chain_offset=off)
        h.gen_sample(q0[off:off + half], verbose=False)
        parts.append(h.q_chain)
    assert np.array_equal(np.concatenate(parts), h1.q_chain)


def test_philox_baseline_shape_statistics():
    """BASELINE config 2 shape (D=100 unit MVN, dt=0.1, L in [5,20)) at 65,536 chains:
    acceptance ~0.99 (case1c reference: 0.9915), post-warm-up moments of N(0, I)."""
    N, D = 65536, 100
    h, _ = _philox_run(N, D, 30, 10)
    assert 0.985 < h.accept_R < 0.997
    x = h.q_chain[:, 1:, :]
    assert np.abs(x.mean(axis=(0, 1))).max() < 0.02
    assert np.abs(x.std(axis=(0, 1)) - 1).max() < 0.02
    lf = h.n_leapfrog
    assert abs(lf / (N * 30) - 12.0) < 0.05          # E[L] = 12 for U{5..19}


def test_fp_modes_agree_statistically():
    N, D = 8192, 100
    he, _ = _philox_run(N, D, 10, 2, fp_mode="exact")
    hf, _ = _philox_run(N, D, 10, 2, fp_mode="fast")
    # same draws, trajectories differ only by FMA rounding: tiny differences everywhere
    np.testing.assert_allclose(he.q_chain, hf.q_chain, rtol=1e-8, atol=1e-8)


def _np_philox(ctr, key):
    """Vectorised NumPy Philox4x32-10 (ctr: (n,4) uint64 words, key: (2,) ints)."""
    c = [ctr[:, i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    M = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = c[0] * np.uint64(0xD2511F53)
        p1 = c[2] * np.uint64(0xCD9E8D57)
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & M, p1 & M, ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & M, p0 & M]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M
        k1 = (k1 + np.uint64(0xBB67AE85)) & M
    return c


def test_philox_normals_match_numpy_box_muller():
    """The in-kernel fp64 Box-Muller (custom ~1-ulp log/sqrt/sincospi on 52-bit uniforms) agrees
    with NumPy's libm-based Box-Muller on the same Philox words to a few ulp (absolute, scaled
    by the radius)."""
    from hmc_amd import _lib as H
    L = H.lib()
    n, npairs, it, seed = 4096, 16, 5, 0x1234_5678_9abc
    out = torch.empty((n, 2 * npairs), dtype=torch.float64, device="cuda")
    H.check(L.hmc_rng_normals(seed, 77, n, it, npairs, out.data_ptr(), None))
    got = out.cpu().numpy().reshape(n, npairs, 2)
    rows = np.repeat(np.arange(n, dtype=np.uint64) + np.uint64(77), npairs)
    ks = np.tile(np.arange(npairs, dtype=np.uint64), n)
    ctr = np.stack([ks, np.full_like(ks, it), rows & np.uint64(0xFFFFFFFF), rows >> np.uint64(32)], axis=1)
    w = _np_philox(ctr, (seed & 0xFFFFFFFF, seed >> 32))
    a = ((w[1] << np.uint64(20)) | (w[0] >> np.uint64(12))).astype(np.float64)   # top 52 bits
    b = ((w[3] << np.uint64(20)) | (w[2] >> np.uint64(12))).astype(np.float64)
    u1 = 1.0 - a * 2.0 ** -52                                                     # (0, 1]
    u2 = b * 2.0 ** -52                                                           # [0, 1)
    r = np.sqrt(-2.0 * np.log(u1))
    z0 = r * np.cos(2 * np.pi * u2)
    z1 = r * np.sin(2 * np.pi * u2)
    ref = np.stack([z0, z1], axis=1).reshape(n, npairs, 2)
    err = np.abs(got - ref) / (r.reshape(n, npairs, 1) + 1e-300)
    assert err.max() < 4e-15, err.max()


@pytest.mark.parametrize("D,thin,wu,gen", [(131, 2, 5, True), (128, 1, 0, False), (200, 3, 7, True),
                                           (1000, 1, 3, False)])
def test_wave_kernel_replay_exact_vs_oracle(D, thin, wu, gen):
    """Wave-per-chain kernel (D > 64): bit-exact q_chain vs the oracle on identical replayed
    streams, incl. odd D, thinning, warm-up 0, general diagonal target (q0, P, M, vector dt)."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    rs = np.random.RandomState(D + thin)
    N, Niter, lo, hi = 3, 30, 3, 11
    if gen:
        q0 = rs.standard_normal(D) * 0.5
        cov0 = np.diag(rs.uniform(0.5, 2.0, D))
        cov_p = np.diag(rs.uniform(0.8, 1.3, D))
        dt = rs.uniform(0.05, 0.15, D)
    else:
        q0, cov0, cov_p, dt = np.zeros(D), np.eye(D), None, 0.1
    tgt = O.MVNTarget(q0, cov0)
    h = HMC_sampler(D, tgt.V, tgt.dVdq, Nchain=N, Niter=Niter, sampler_type="Random", L_low=lo, L_high=hi, dt=dt,
                    thin_rate=thin, warm_up_num=wu, cov_p=cov_p, target=MVNTarget(q0, cov0))
    q_start = rs.standard_normal((N, D))
    np.random.seed(D)
    h.gen_sample(q_start, verbose=False)
    np.random.seed(D)
    ref = O.gen_sample_random(O.HMCCore(tgt, dt, cov_p), q_start, N, Niter, wu, thin, lo, hi,
                              O.LiveDraws(D, h.cov_p))
    assert np.array_equal(h.q_chain, ref["q_chain"])
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-12)
    np.testing.assert_allclose(h.dE_chain[:, :, 0], ref["dE_chain"], rtol=1e-8, atol=1e-10)
    assert h.accept_R == ref["accept_R"]
    assert h.N_total_steps == ref["N_total_steps"]


DENSE_FIXTURES = ["f3_case3c_small.npz", "f3b_case3a.npz", "f11_case5_unstable.npz",
                  "f12_dense_covp.npz"]   # f12: full (non-diagonal) cov_p, Q3 (samplers.py:352-356, :825-839)


@pytest.mark.parametrize("fx", DENSE_FIXTURES)
@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_dense_replay_matches_reference(fx, fp_mode):
    """Correlated targets (dense inv(cov0), f64 MFMA gradient): same draws as the reference,
    so the accept/reject sequence is identical and the states agree to round-off (the MFMA
    k-ordered sums differ from BLAS dgemv in the last bits).  Tolerance: q_chain 1e-9 abs/rel,
    E 1e-10 rel, R-hat / std 1e-6 rel (north-star contract)."""
    g = load_golden(fx)
    m = g["meta"]
    h = _run_replay(g, fp_mode)
    assert h.accept_R == float(g["accept_R"])
    if m["warm_up"] > 0:
        assert h.accept_R_warm_up == float(g["accept_R_warm_up"])
    assert h.N_total_steps == int(g["N_total_steps"])
    np.testing.assert_allclose(h.q_chain, g["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], g["E_chain"], rtol=1e-10)
    h.compute_convergence_stats()
    np.testing.assert_allclose(h.R_q, g["R_q"], rtol=1e-6)
    from hmc_amd.diagnostics import per_dim_mean_std
    mean, std = per_dim_mean_std(h.q_chain_device)
    np.testing.assert_allclose(std, g["std"], rtol=1e-6)


@pytest.mark.parametrize("D,rho", [(100, 0.95), (37, 0.5), (128, 0.9)])
def test_dense_philox_statistics(D, rho):
    """Philox mode, dense target at scale, chains started IN the stationary law N(0, Sigma):
    HMC leaves it invariant, so after any number of iterations the per-dim variances are 1
    and corr(q0, q1) = rho (independent of mixing speed); results are deterministic."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    cov = O.mvn_cov(D, rho)
    N = 8192
    q0 = np.random.RandomState(D).standard_normal((N, D)) @ np.linalg.cholesky(cov).T

    def run():
        h = HMC_sampler(D, None, None, Nchain=N, Niter=12, sampler_type="Random", L_low=5, L_high=20, dt=0.1,
                        warm_up_num=2, target=MVNTarget(np.zeros(D), cov), rng="philox", seed=3, fp_mode="fast")
        h.gen_sample(q0, verbose=False)
        return h
    h = run()
    x = h.q_chain[:, 1:, :]
    last = x[:, -1, :]                                  # one draw per chain: independent samples
    assert np.abs(last.var(axis=0) - 1).max() < 6 * np.sqrt(2 / N)
    assert abs(np.corrcoef(last[:, 0], last[:, 1])[0, 1] - rho) < 6 * (1 - rho ** 2) / np.sqrt(N)
    assert 0.5 < h.accept_R <= 1.0
    h2 = run()
    assert np.array_equal(h.q_chain, h2.q_chain)


@pytest.mark.parametrize("rng", ["philox", "replay"])
@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_dense_L_ordered_tiles_identical(rng, fp_mode):
    """L-ordered MFMA tiles (chains counting-sorted by trajectory length every iteration) only
    move chains between lanes: every output is bit-identical to the chain-ordered launch.
    N = 1000 leaves a ragged last tile; the replay streams include L at both range ends."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    D, N, Niter, wu = 100, 1000, 7, 2
    cov = O.mvn_cov(D, 0.95)
    rs = np.random.RandomState(11)
    q_start = rs.standard_normal((N, D)) @ np.linalg.cholesky(cov).T
    streams = (rs.standard_normal((N, D)), rs.standard_normal((N, Niter, D)),
               rs.randint(5, 20, size=(N, Niter)).astype(np.int32), np.log(rs.random_sample((N, Niter))))
    out = []
    for order in (True, False):
        eng = RandomEngine(MVNTarget(np.zeros(D), cov), N, Niter, wu, 1, 5, 20, 0.1, rng=rng, seed=9,
                           fp_mode=fp_mode, order_tiles=order)
        assert (eng._order is not None) == order
        if rng == "replay":
            eng.set_replay(*streams)
        eng.init(q_start)
        eng.run(1, 4)
        eng.run(4, Niter + 1)
        torch.cuda.synchronize()
        out.append([eng.q_chain.cpu().numpy(), eng.E_chain.cpu().numpy(), eng.dE_chain.cpu().numpy(),
                    eng.q.cpu().numpy(), eng.read_counters()])
    for a, b in zip(*out):
        assert np.array_equal(a, b)


def test_dense_mass_matrix_rows_and_stationarity():
    """Full cov_p (Q3: K = p.inv(cov_p).p/2, p ~ N(0, cov_p), kick by inv(cov_p).dVdq, drift by
    p).  Row API vs the oracle's HMCCore (samplers.py:811-839) to round-off; Philox chains
    started in N(0, Sigma) stay there (the reference's proposal is a reversible volume-preserving
    map with an exact MH correction, so the target is invariant) and are deterministic."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    import make_golden_shapes as S
    D, rho = 12, 0.6
    cov, cov_p = O.mvn_cov(D, rho), S.dense_cov_p(D)
    tgt = O.MVNTarget(np.zeros(D), cov)
    core = O.HMCCore(tgt, 0.1, cov_p)
    rs = np.random.RandomState(5)
    P, Q = rs.standard_normal((4, D)), rs.standard_normal((4, D))
    h = HMC_sampler(D, tgt.V, tgt.dVdq, Nchain=2, Niter=1, sampler_type="Random", L_low=1, L_high=2, dt=0.1,
                    cov_p=cov_p, target=MVNTarget(np.zeros(D), cov))
    pn, qn = h.leap_frog(P, Q)
    for i in range(4):
        pr, qr = core.leap_frog(P[i], Q[i])
        np.testing.assert_allclose(pn[i], pr, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(qn[i], qr, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(h.E(Q[i], P[i]), core.E(Q[i], P[i]), rtol=1e-12)
    N = 8192
    q0 = rs.standard_normal((N, D)) @ np.linalg.cholesky(cov).T

    def run():
        s = HMC_sampler(D, None, None, Nchain=N, Niter=10, sampler_type="Random", L_low=5, L_high=20, dt=0.1,
                        warm_up_num=2, cov_p=cov_p, target=MVNTarget(np.zeros(D), cov), rng="philox", seed=3,
                        fp_mode="fast")
        s.gen_sample(q0, verbose=False)
        return s
    a = run()
    last = a.q_chain[:, -1, :]
    assert np.abs(last.var(axis=0) - 1).max() < 6 * np.sqrt(2 / N)
    assert abs(np.corrcoef(last[:, 0], last[:, 1])[0, 1] - rho) < 6 * (1 - rho ** 2) / np.sqrt(N)
    assert 0.05 < a.accept_R < 1.0
    assert np.array_equal(a.q_chain, run().q_chain)


def test_dense_checkpoint_resume_bitexact(tmp_path):
    """Dense L-ordered engine (gradient cache in the workspace): checkpoint after iteration 3,
    resume in a fresh engine, identical to the uninterrupted run; re-initialising q invalidates
    the cache (the next launch recomputes every gradient)."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    D, N, Niter = 100, 777, 7
    cov = O.mvn_cov(D, 0.9)
    q0 = np.random.RandomState(5).standard_normal((N, D)) @ np.linalg.cholesky(cov).T

    def make():
        e = RandomEngine(MVNTarget(np.zeros(D), cov), N, Niter, 1, 1, 5, 20, 0.1, rng="philox", seed=21,
                         fp_mode="fast")
        e.init(q0)
        return e
    ref = make()
    for a in range(1, Niter + 1):
        ref.run(a, a + 1)
    a_ = make()
    for a in range(1, 4):
        a_.run(a, a + 1)
    path = str(tmp_path / "dense.npz")
    a_.save(path, 4)
    b = RandomEngine(MVNTarget(np.zeros(D), cov), N, Niter, 1, 1, 5, 20, 0.1, rng="philox", seed=21, fp_mode="fast")
    assert b.restore(path) == 4
    for a in range(4, Niter + 1):
        b.run(a, a + 1)
    torch.cuda.synchronize()
    assert torch.equal(b.q, ref.q) and torch.equal(b.q_chain, ref.q_chain) and torch.equal(b.E_chain, ref.E_chain)
    a_.init(q0)                                   # same start again: same chains as ref's first iterations
    for a in range(1, Niter + 1):
        a_.run(a, a + 1)
    torch.cuda.synchronize()
    assert torch.equal(a_.q_chain, ref.q_chain)
