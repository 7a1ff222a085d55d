"""NUTS beyond the MFMA tree kernel's register budget (hmc_nuts_big.hip): dense targets with
D > 128, which the reference's NUTS takes through np.dot at any D (samplers.py:495-808, :835-837).

Replay mode vs the oracle (oracle/hmc_oracle.py restating gen_sample_NUTS) on the same momenta
and the same per-chain tape of directions / uniforms: identical leapfrog and instability counts,
q_chain within 1e-9, E within 1e-10 relative (GEMV sums in k order vs BLAS).  Philox mode: the
stationary law, determinism and shard invariance (draws keyed by the global chain id)."""
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


CASES = [
    # D, rho, q0 scale, Nchain, Niter, wu, thin, dt, d_max, diag cov_p, dt vector, on_dmax
    (136, 0.9, 0.0, 3, 10, 1, 1, 0.1, 9, False, False, "raise"),
    (300, 0.5, 0.5, 2, 4, 0, 2, 0.15, 8, True, True, "break"),
    (160, 0.99, 0.0, 3, 4, 0, 1, 0.9, 6, False, False, "break"),     # large dt: |E - E0| > 1000 guard
    (129, 0.3, 0.0, 5, 6, 2, 1, 0.02, 3, False, False, "break"),     # d_max reached every iteration
    (144, 0.8, 0.3, 40, 3, 1, 1, 0.2, 6, False, False, "break"),     # lockstep blocks: slots take 2 chains
    (330, 0.6, 0.0, 2, 3, 0, 1, 0.2, 5, False, False, "break"),      # D > 320: the per-chain kernel
]


def _case(case):
    D, rho, qs, N, Niter, wu, thin, dt, d_max, diag_p, dtvec, on_dmax = case
    rs = np.random.RandomState(2000 + D)
    cov = O.mvn_cov(D, rho) if rho > 0 else np.eye(D)
    q0 = rs.standard_normal(D) * qs
    cov_p = np.diag(rs.uniform(0.5, 2.0, D)) if diag_p else None
    dts = rs.uniform(0.5, 1.0, D) * dt if dtvec else dt
    q_start = q0 + rs.standard_normal((N, D)) * 1.2
    scale = np.sqrt(np.diag(cov_p)) if diag_p else np.ones(D)
    p0 = rs.standard_normal((N, D)) * scale
    P = rs.standard_normal((N, Niter, D)) * scale
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))   # int(v) = direction, v = uniform
    return cov, q0, cov_p, dts, q_start, p0, P, tape


@pytest.mark.parametrize("case", CASES, ids=[f"D{c[0]}_rho{c[1]}_dt{c[7]}_dmax{c[8]}" for c in CASES])
@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
def test_nuts_large_D_vs_oracle(case, fp_mode):
    from hmc_amd import _lib as H
    from hmc_amd.engine import NutsEngine
    from hmc_amd.target import MVNTarget
    D, rho, qs, N, Niter, wu, thin, dt, d_max, diag_p, dtvec, on_dmax = case
    cov, q0, cov_p, dts, q_start, p0, P, tape = _case(case)
    tgt = FastMVN(q0, cov)
    ref = O.gen_sample_nuts(O.HMCCore(tgt, dts, cov_p), q_start, N, Niter, wu, thin, d_max,
                            O.ReplayDraws(p0, P, tape=tape.copy()), on_dmax=on_dmax)
    eng = NutsEngine(MVNTarget(q0, cov, logdet_const=tgt.c), N, Niter, wu, thin, d_max, dts, cov_p=cov_p,
                     rng="replay", fp_mode=fp_mode, on_dmax=on_dmax)
    eng.set_replay(p0, P, tape)
    eng.init(q_start)
    eng.run(1, 3)                                 # two launches: the tape cursors persist between them
    eng.run(3, Niter + 1)
    torch.cuda.synchronize()
    c = eng.read_counters()
    assert int(c[H.CNT_OOB_REJECT]) == 0
    assert int(c[H.CNT_LEAPFROG]) == ref["n_leapfrog"]
    assert int(c[H.CNT_UNSTABLE]) == ref["n_unstable"]
    if on_dmax == "raise":
        assert int(c[H.CNT_DMAX]) == 0
    np.testing.assert_allclose(eng.q_chain.cpu().numpy(), ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.E_chain.cpu().numpy(), ref["E_chain"], rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(eng.dE_chain.cpu().numpy(), ref["dE_chain"], rtol=1e-8, atol=1e-9)
    if case[0] == 160:
        assert ref["n_unstable"] > 0              # the case exercises the guard
    if case[0] == 129:
        assert int(c[H.CNT_DMAX]) == N * Niter    # and this one the d_max break


def test_nuts_large_D_through_sampler():
    """The drop-in surface: HMC_sampler(sampler_type='NUTS') at D = 200 with the reference's
    accounting (N_total_steps, accept_R = 1) on replayed draws vs the oracle."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    D, N, Niter, wu, d_max, dt = 200, 2, 4, 1, 8, 0.1
    rs = np.random.RandomState(5)
    cov = O.mvn_cov(D, 0.8)
    q_start = rs.standard_normal((N, D))
    p0, P = rs.standard_normal((N, D)), rs.standard_normal((N, Niter, D))
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))
    tgt = FastMVN(np.zeros(D), cov)
    ref = O.gen_sample_nuts(O.HMCCore(tgt, dt), q_start, N, Niter, wu, 1, d_max,
                            O.ReplayDraws(p0, P, tape=tape.copy()))
    h = HMC_sampler(D, None, None, Nchain=N, Niter=Niter, thin_rate=1, warm_up_num=wu, sampler_type="NUTS",
                    dt=dt, d_max=d_max, target=MVNTarget(np.zeros(D), cov, logdet_const=tgt.c), rng="replay")
    h.set_nuts_replay(p0, P, tape)
    h.gen_sample(q_start, verbose=False)
    assert h.n_leapfrog == ref["n_leapfrog"]
    assert h.N_total_steps == ref["N_total_steps"]
    assert h.accept_R == 1.0
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)


def test_nuts_large_D_philox_stationary_and_shards():
    """Chains started in N(0, Sigma) stay there (per-dim variance 1, corr rho); runs repeat bit for
    bit, and two shards (chain_offset) reproduce the one-batch run (Philox keyed by global chain)."""
    from hmc_amd.engine import NutsEngine
    from hmc_amd.target import MVNTarget
    D, rho, N, Niter = 160, 0.6, 1024, 3
    cov = O.mvn_cov(D, rho)
    qs = np.random.RandomState(4).standard_normal((N, D)) @ np.linalg.cholesky(cov).T
    tgt = MVNTarget(np.zeros(D), cov)

    def run(lo, hi):
        e = NutsEngine(tgt, hi - lo, Niter, 1, 1, 10, 0.2, rng="philox", seed=11, chain_offset=lo,
                       on_dmax="break")
        e.init(qs[lo:hi])
        e.run(1, Niter + 1)
        torch.cuda.synchronize()
        return e.q_chain.cpu().numpy(), e.read_counters()
    qc, cnt = run(0, N)
    last = qc[:, -1, :]
    assert np.abs(last.var(axis=0).mean() - 1) < 6 * np.sqrt(2 / (N * D)) + 0.02
    assert abs(np.corrcoef(last[:, 0], last[:, 1])[0, 1] - rho) < 6 * (1 - rho ** 2) / np.sqrt(N) + 0.02
    assert np.isfinite(qc).all()
    assert np.array_equal(qc, run(0, N)[0])
    a, b = run(0, 400), run(400, N)
    assert np.array_equal(np.concatenate([a[0], b[0]]), qc)
    from hmc_amd import _lib as H
    res = [i for i in range(H.NCOUNTERS) if i != H.CNT_LEAPFROG_SQ]   # (slot 3: block steps, a schedule statistic)
    assert (a[1][res] + b[1][res] == cnt[res]).all()


@pytest.mark.parametrize("fp_mode", ["exact", "fast"])
@pytest.mark.parametrize("D", [136, 300, 330])
def test_nuts_large_D_full_cov_p_vs_oracle(D, fp_mode):
    """A full (non-diagonal) cov_p above D = 128 (samplers.py:352-356, :811-839 through
    gen_sample_NUTS): at D = 136 and 300 the lockstep kernel's block GEMMs (round 6: P x, the kick
    inv_cov_p . P x, and inv_cov_p p for K), at D = 330 the per-chain kernel's GEMVs, on replayed
    draws vs the oracle; plus Philox determinism."""
    import make_golden_shapes as S
    from hmc_amd import _lib as H
    from hmc_amd.engine import NutsEngine
    from hmc_amd.target import MVNTarget
    N, Niter, wu, dt, d_max = 3, 4, 1, 0.15, 7
    rs = np.random.RandomState(90 + D)
    cov, cov_p = O.mvn_cov(D, 0.6), S.dense_cov_p(D)
    C = np.linalg.cholesky(cov_p)
    q_start = rs.standard_normal((N, D)) * 1.2
    p0 = rs.standard_normal((N, D)) @ C.T
    P = rs.standard_normal((N, Niter, D)) @ C.T
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))
    tgt = FastMVN(np.zeros(D), cov)
    ref = O.gen_sample_nuts(O.HMCCore(tgt, dt, cov_p), q_start, N, Niter, wu, 1, d_max,
                            O.ReplayDraws(p0, P, tape=tape.copy()), on_dmax="break")
    eng = NutsEngine(MVNTarget(np.zeros(D), cov, logdet_const=tgt.c), N, Niter, wu, 1, d_max, dt, cov_p=cov_p,
                     rng="replay", fp_mode=fp_mode, on_dmax="break")
    eng.set_replay(p0, P, tape)
    eng.init(q_start)
    eng.run(1, Niter + 1)
    torch.cuda.synchronize()
    c = eng.read_counters()
    assert int(c[H.CNT_LEAPFROG]) == ref["n_leapfrog"]
    assert int(c[H.CNT_UNSTABLE]) == ref["n_unstable"]
    np.testing.assert_allclose(eng.q_chain.cpu().numpy(), ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.E_chain.cpu().numpy(), ref["E_chain"], rtol=1e-10, atol=1e-10)
    if D != 136 or fp_mode != "fast":
        return
    # Philox (p = C z): finite and repeatable.  No stationarity check here: the reference's NUTS
    # with a cov_p other than the identity (Q3 leapfrog, Q11 ratio) does not keep N(0, Sigma) --
    # the oracle itself, on np.random draws at D = 8, 1,500 chains, 3 iterations, dt = 0.2: mean
    # per-dim variance 1.38 (full cov_p), 1.30 (its diagonal), 1.05 (identity) -- and the replay
    # parity above pins this kernel to the reference's behaviour instead.
    N2 = 256
    qs = np.random.RandomState(4).standard_normal((N2, D)) @ np.linalg.cholesky(cov).T

    def run():
        e = NutsEngine(MVNTarget(np.zeros(D), cov), N2, 3, 1, 1, 8, 0.2, cov_p=cov_p, rng="philox", seed=6,
                       on_dmax="break")
        e.init(qs)
        e.run(1, 4)
        torch.cuda.synchronize()
        return e.q_chain.cpu().numpy()
    qc = run()
    assert np.isfinite(qc).all()
    assert not np.array_equal(qc[:, -1, :], qc[:, 0, :])
    assert np.array_equal(qc, run())


def test_nuts_large_D_streaming_and_resume(tmp_path):
    """The large-D NUTS path under the surface's streaming mode (HMC_sampler(store_chain=False):
    E_chain identical to the stored run, R-hat equal to the oracle's convergence_stats on the stored
    q_chain), and a checkpoint at iteration 7 resumed in a fresh engine: bit-identical to the
    uninterrupted run (Philox keyed by iteration; the workspace travels in the checkpoint)."""
    from hmc_amd.engine import NutsEngine
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    D, N, Niter, wu = 144, 16, 40, 8
    cov = O.mvn_cov(D, 0.5)
    tgt = MVNTarget(np.zeros(D), cov)
    q_start = np.random.RandomState(8).standard_normal((N, D))
    kw = dict(Nchain=N, Niter=Niter, sampler_type="NUTS", dt=0.2, warm_up_num=wu, rng="philox", seed=5,
              fp_mode="fast", iters_per_launch=8, target=tgt, d_max=10)
    full = HMC_sampler(D, None, None, **kw)
    full.gen_sample(q_start, verbose=False)
    h = HMC_sampler(D, None, None, store_chain=False, stream_tmax=16, stream_feed=16, **kw)
    h.gen_sample(q_start, verbose=False)
    assert h.q_chain is None
    assert np.array_equal(h.E_chain, full.E_chain)
    h.compute_convergence_stats()
    R_ref, _ = O.convergence_stats(full.q_chain[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(h.R_q, R_ref, rtol=1e-10)

    def make():
        return NutsEngine(tgt, N, 12, 2, 1, 10, 0.2, rng="philox", seed=3, on_dmax="break")
    ref = make()
    ref.init(q_start)
    ref.run(1, 13)
    a = make()
    a.init(q_start)
    a.run(1, 7)
    path = str(tmp_path / "nuts_big.npz")
    a.save(path, 7)
    b = make()
    it = b.restore(path)
    assert it == 7
    b.run(it, 13)
    torch.cuda.synchronize()
    assert torch.equal(b.q, ref.q)
    assert torch.equal(b.q_chain, ref.q_chain)
    np.testing.assert_array_equal(b.read_counters(), ref.read_counters())


@pytest.mark.parametrize("D,full", [(200, False), (136, True), (330, True)])
def test_nuts_large_D_deep_tree_vs_oracle(D, full):
    """Trees of more than 2^15 points above D = 128 (advisor r05: d_max was raised to 30 on every
    NUTS kernel, but only the D = 2 tree kernel ran a tree deeper than 15): the lockstep kernel at
    D = 200 (diagonal cov_p) and D = 136 (full cov_p), the per-chain kernel at D = 330 (full cov_p),
    d_max = 18, one chain, a step small enough that both ends turn only after 2^15 points.  Leapfrog
    counts, q_chain and E equal the oracle's on the same replayed draws; no d_max hit."""
    import make_golden_shapes as S
    from hmc_amd import _lib as H
    from hmc_amd.engine import NutsEngine
    from hmc_amd.target import MVNTarget
    N, Niter, d_max = 1, 1, 18
    dt = 5e-5 if not full else 1e-4
    rs = np.random.RandomState(70 + D)
    cov = np.eye(D)
    cov_p = S.dense_cov_p(D) if full else None
    C = np.linalg.cholesky(cov_p) if full else np.eye(D)
    q_start = rs.standard_normal((N, D))
    p0 = rs.standard_normal((N, D)) @ C.T
    P = rs.standard_normal((N, Niter, D)) @ C.T
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * ((1 << 17) + d_max + 2)))
    tgt = FastMVN(np.zeros(D), cov)
    ref = O.gen_sample_nuts(O.HMCCore(tgt, dt, cov_p), q_start, N, Niter, 0, 1, d_max,
                            O.ReplayDraws(p0, P, tape=tape.copy()), on_dmax="break")
    assert ref["n_leapfrog"] > 1 << 15, ref["n_leapfrog"]
    eng = NutsEngine(MVNTarget(np.zeros(D), cov, logdet_const=tgt.c), N, Niter, 0, 1, d_max, dt, cov_p=cov_p,
                     rng="replay", fp_mode="exact", on_dmax="break")
    eng.set_replay(p0, P, tape)
    eng.init(q_start)
    eng.run(1, Niter + 1)
    torch.cuda.synchronize()
    c = eng.read_counters()
    assert int(c[H.CNT_DMAX]) == 0 and int(c[H.CNT_OOB_REJECT]) == 0
    assert int(c[H.CNT_LEAPFROG]) == ref["n_leapfrog"]
    np.testing.assert_allclose(eng.q_chain.cpu().numpy(), ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.E_chain.cpu().numpy(), ref["E_chain"], rtol=1e-10, atol=1e-10)
