"""The production (Philox) kernel instantiations pinned to the oracle.

bench.py times `k_wave_iters_k1<EXACT=false, GEN=false, REPLAY=false, FULL=false>` (D <= 128:
in-kernel Philox4x32-10 draws through the momentum ring, FAST integrator, no capture hooks),
`k_wave_iters<K=2/4/8, ..., FULL=false>` (D > 128, BASELINE config 4: per-lane momentum draws,
streaming window), the dense L-ordered-tile kernel and the NUTS kernel in Philox mode.  Here every
random number those kernels consume is regenerated on the HOST from the same counters
(tests/philox_host.py: NumPy Philox4x32-10 and the table-driven Box-Muller restated) and replayed
through the oracle (oracle/hmc_oracle.py, which restates samplers.py:387-491 / :495-808):
  * momentum of iteration >= 1: the table Box-Muller (hmc_device.hpp::normal_pair_tab) restated in
    NumPy; the initial momentum (iteration 0, samplers.py:415) plain Box-Muller
    (hmc_device.hpp::normal_pair); test_table_normals_match_kernel pins the restatement to the
    kernels' generator (C-ABI debug entry hmc_rng_normals) to 1e-13;
  * trajectory length L (samplers.py:441) and MH log-uniform (:461): Philox block
    (0x80000000, iteration, chain lo, chain hi): L = L_low + (x * (L_high - L_low)) >> 32,
    u = ((w << 21) | (z >> 11)) * 2^-53, log u (NumPy log; the kernel's fast_log is within 1 ulp);
  * NUTS directions / uniforms (:608, :750, :773): the k-th draw of an iteration is the block
    (0x80000000 + k, iteration, chain): direction = x & 1, uniform = u53(z, w).
Assertions: identical accept counts and leapfrog counts, q_chain within 1e-9 (FAST integrator
and MFMA sums vs the reference's arithmetic), E within 1e-10 relative.
"""
import numpy as np
import pytest
import torch

from oracle import hmc_oracle as O
from philox_host import KDRAW, bm_pair, host_L_lnu, table_normals, u53, wave_momenta, words

pytestmark = pytest.mark.gpu


def gpu_normals(seed, chain0, n, it, npairs):
    """The kernels' table-driven normals for (chain0 + row, iteration it, slots 0..npairs-1)."""
    from hmc_amd import _lib as H
    out = torch.empty((n, 2 * npairs), dtype=torch.float64, device="cuda")
    H.check(H.lib().hmc_rng_normals(seed, chain0, n, it, npairs, out.data_ptr(), None), "hmc_rng_normals")
    return out.cpu().numpy()


@pytest.mark.parametrize("npairs,chain0,it", [(50, 0, 1), (500, 1 << 33, 17), (64, 12345, 999)])
def test_table_normals_match_kernel(npairs, chain0, it):
    """The host restatement of the table Box-Muller equals the kernels' generator to 1e-13
    (both are ~1-ulp evaluations of the same function of the same Philox words)."""
    seed = 0x1234_5678_9ABC
    g = gpu_normals(seed, chain0, 96, it, npairs)
    h = table_normals(seed, chain0, 96, it, npairs)
    assert np.all(np.isfinite(g))
    np.testing.assert_allclose(g, h, rtol=0, atol=1e-13)


def dense_slot_index(D):
    """Dense/NUTS kernels: dims h + 4m (h < 4), pairs (m, m+1) for even m in slot h + 4m:
    dim d -> (slot, which of the pair)."""
    d = np.arange(D)
    h, m = d % 4, d // 4
    return h + 4 * (m - (m & 1)), m & 1


def dense_momenta(seed, N, D, niter, table=True):
    slot, which = dense_slot_index(D)
    gcs = np.arange(N, dtype=np.uint64)
    z = bm_pair(words(slot[None, :], 0, gcs[:, None], seed))
    p0 = np.where(which[None, :] == 0, z[0], z[1])
    P = np.empty((N, niter, D))
    for it in range(1, niter + 1):
        if table:
            g = table_normals(seed, 0, N, it, D)
            P[:, it - 1] = g[:, 2 * slot + which]
        else:
            z = bm_pair(words(slot[None, :], it, gcs[:, None], seed))
            P[:, it - 1] = np.where(which[None, :] == 0, z[0], z[1])
    return p0, P


class FastMVN(O.MVNTarget):
    """Oracle target with V evaluated as 0.5 (logdet const + x.P.x) instead of scipy's eigh-based
    logpdf on every call (same value to ~1e-14; keeps the larger NUTS cases fast)."""

    def __init__(self, q0, cov0):
        super().__init__(q0, cov0)
        D = self.q0.size
        self.c = D * np.log(2 * np.pi) + np.linalg.slogdet(self.cov0)[1]

    def V(self, q):
        x = q - self.q0
        return 0.5 * (self.c + x @ (self.inv_cov0 @ x))


@pytest.mark.parametrize("fp_mode", ["fast", "exact"])
def test_wave_production_kernel_vs_oracle(fp_mode):
    """The benchmarked instantiation (D=100 unit MVN, Philox, one fused launch, no capture):
    64 chains x 30 iterations vs the oracle on the host-regenerated draws."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    N, D, Niter, wu, seed = 64, 100, 30, 5, 0x5EED_0001
    rs = np.random.RandomState(7)
    q_start = rs.standard_normal((N, D)) * np.sqrt(2.0)
    h = HMC_sampler(D, None, None, Nchain=N, Niter=Niter, sampler_type="Random", L_low=5, L_high=20, dt=0.1,
                    warm_up_num=wu, target=MVNTarget(np.zeros(D), np.eye(D)), rng="philox", seed=seed,
                    fp_mode=fp_mode)
    h.gen_sample(q_start, verbose=False)
    # EXACT asserts the integrator bit for bit, so it replays the generator's own output (read back
    # through hmc_rng_normals, itself pinned to the host restatement by test_table_normals_match_kernel);
    # FAST replays the host restatement
    p0, P = wave_momenta(seed, N, D, Niter, normals=gpu_normals if fp_mode == "exact" else table_normals)
    L, lnu = host_L_lnu(seed, np.arange(N, dtype=np.uint64), Niter, 5, 20)
    ref = O.gen_sample_random(O.HMCCore(O.MVNTarget(np.zeros(D), np.eye(D)), 0.1), q_start, N, Niter, wu, 1, 5, 20,
                              O.ReplayDraws(p0, P, L, lnu))
    assert h._acc == ref["accept_count"] and h._acc_wu == ref["accept_count_warm_up"]
    assert h.accept_R == ref["accept_R"] and h.accept_R_warm_up == ref["accept_R_warm_up"]
    assert h.n_leapfrog == ref["n_leapfrog"] == int(L.sum())
    assert h.N_total_steps == ref["N_total_steps"]
    if fp_mode == "exact":
        assert np.array_equal(h.q_chain, ref["q_chain"])
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-10)


def test_wave_production_window_vs_oracle():
    """bench.py's storage path: every row written into a circular window of R rows (row r at
    slot r % R) over several fused launches; the window then holds the oracle's last R rows."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, D, S, launches, seed = 96, 100, 8, 5, 11
    Niter = S * launches
    wu = S + 1                                   # rows 0 .. (launches-1)*S - 1 after warm-up
    R = 8
    eng = RandomEngine(MVNTarget(np.zeros(D), np.eye(D)), N, Niter, wu, 1, 5, 20, 0.1, rng="philox", seed=seed,
                       fp_mode="fast", store_chain=False)
    win = torch.zeros((N, R, D), dtype=torch.float64, device=eng.device)
    eng.set_chain_window(win, 0)
    q_start = np.random.RandomState(3).standard_normal((N, D))
    eng.init(q_start)
    for k in range(launches):
        eng.run(1 + k * S, 1 + (k + 1) * S)
    torch.cuda.synchronize()
    p0, P = wave_momenta(seed, N, D, Niter)
    L, lnu = host_L_lnu(seed, np.arange(N, dtype=np.uint64), Niter, 5, 20)
    ref = O.gen_sample_random(O.HMCCore(O.MVNTarget(np.zeros(D), np.eye(D)), 0.1), q_start, N, Niter, wu, 1, 5, 20,
                              O.ReplayDraws(p0, P, L, lnu))
    rows = ref["q_chain"].shape[1]
    assert rows % R == 0
    np.testing.assert_allclose(win.cpu().numpy(), ref["q_chain"][:, rows - R:], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.E_chain.cpu().numpy(), ref["E_chain"], rtol=1e-10)
    c = eng.read_counters()
    from hmc_amd import _lib as H
    assert int(c[H.CNT_LEAPFROG]) == ref["n_leapfrog"]


class UnitCore(O.HMCCore):
    """oracle HMCCore for an identity precision and mass: np.dot(I, g) == g exactly, so the
    half kicks are written without the D x D products (same arithmetic, D=1000 stays fast)."""

    def leap_frog(self, p_old, q_old):              # samplers.py:831-839 with inv_cov_p = inv_cov0 = I
        p_half = p_old - self.dt * (q_old - self.t.q0) / 2.
        q_new = q_old + self.dt * p_half
        p_new = p_half - self.dt * (q_new - self.t.q0) / 2.
        return p_new, q_new


class UnitMVN(FastMVN):
    def __init__(self, D):
        self.q0 = np.zeros(D)
        self.c = D * np.log(2 * np.pi)

    def V(self, q):
        x = q - self.q0
        return 0.5 * (self.c + x @ x)


@pytest.mark.parametrize("D", [129, 200, 300, 1000])
def test_wave_kgt1_production_streaming_vs_oracle(D):
    """BASELINE config 4's benchmarked instance, k_wave_iters<K = 2, 2, 4, 8, FAST, Philox,
    FULL=false> (per-lane wave_momentum draws, D > 128; odd D = 129 included), driven the way
    bench.py --stream-diag drives it: RandomEngine.run_streaming (circular q_chain window, several
    fused launches, the streaming statistics fed every `feed` iterations, tmax = 16).  The oracle
    replays the host-regenerated draws: accept and leapfrog counts exact, q and E_chain to
    1e-9 / 1e-10, streamed R-hat equal to the oracle's convergence_stats (utils.py:77-126) to
    1e-10 and ESS wherever the reference reads no lag beyond tmax."""
    from hmc_amd import _lib as H
    from hmc_amd.diagnostics import StreamingDiagnostics
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, Niter, wu, seed, step, feed = 48, 24, 3, 0xC4_0000 + D, 4, 8
    eng = RandomEngine(MVNTarget(np.zeros(D), np.eye(D)), N, Niter, wu, 1, 5, 20, 0.1, rng="philox", seed=seed,
                       fp_mode="fast", store_chain=False)
    q_start = np.random.RandomState(D).standard_normal((N, D)) * np.sqrt(2.0)
    eng.init(q_start)
    sd = StreamingDiagnostics(N, D, eng.L_chain - 1, tmax=16)
    eng.run_streaming(sd, 1, Niter + 1, step, feed=feed)
    R, neff = sd.finish()
    p0, P = wave_momenta(seed, N, D, Niter)
    L, lnu = host_L_lnu(seed, np.arange(N, dtype=np.uint64), Niter, 5, 20)
    ref = O.gen_sample_random(UnitCore(UnitMVN(D), 0.1), q_start, N, Niter, wu, 1, 5, 20,
                              O.ReplayDraws(p0, P, L, lnu))
    c = eng.read_counters()
    assert int(c[H.CNT_ACCEPT]) == ref["accept_count"] and int(c[H.CNT_ACCEPT_WU]) == ref["accept_count_warm_up"]
    assert int(c[H.CNT_LEAPFROG]) == ref["n_leapfrog"] == int(L.sum())
    np.testing.assert_allclose(eng.q.cpu().numpy(), ref["q_chain"][:, -1], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(eng.E_chain.cpu().numpy(), ref["E_chain"], rtol=1e-10)
    R_ref, neff_ref = O.convergence_stats(ref["q_chain"][:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    from test_gpu_stream import _lags_needed
    ok = _lags_needed(ref["q_chain"][:, 1:, :]) <= 16
    assert ok.sum() >= 5
    np.testing.assert_allclose(neff[ok], neff_ref[ok], rtol=1e-10)


def test_wave_c4_shard_full_shape():
    """One config-4 shard at its benchmarked size: 131,072 chains x D = 1000 (K = 8), Philox,
    streaming window and statistics, started in the stationary law N(0, I).  Acceptance near the
    c4 bench's 0.973, leapfrogs per iteration 12, the law preserved, and the two halves run as
    separate shards (chain_offset) bit-identical to the whole, streamed sums included."""
    from hmc_amd import _lib as H
    from hmc_amd.diagnostics import StreamingDiagnostics
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, D, Niter, wu, step = 131072, 1000, 30, 1, 10
    g = torch.Generator(device="cuda").manual_seed(44)
    qs = torch.randn((N, D), dtype=torch.float64, device="cuda", generator=g)

    def run(lo, hi):
        eng = RandomEngine(MVNTarget(np.zeros(D), np.eye(D)), hi - lo, Niter, wu, 1, 5, 20, 0.1, rng="philox",
                           seed=0xC4, fp_mode="fast", chain_offset=lo, store_chain=False)
        eng.init(qs[lo:hi].contiguous())
        sd = StreamingDiagnostics(hi - lo, D, eng.L_chain - 1, tmax=16)
        eng.run_streaming(sd, 1, Niter + 1, step, feed=step)
        torch.cuda.synchronize()
        out = (eng.q.clone(), eng.read_counters(), sd)
        del eng
        return out

    q_all, c_all, sd_all = run(0, N)
    acc = c_all[H.CNT_ACCEPT] / (N * Niter)
    assert abs(acc - 0.973) < 0.01, acc
    assert abs(c_all[H.CNT_LEAPFROG] / (N * Niter) - 12.0) < 0.02
    x = q_all.cpu().numpy()
    assert np.abs(x.mean(axis=0)).max() < 6 / np.sqrt(N)
    assert np.abs(x.var(axis=0) - 1).max() < 6 * np.sqrt(2 / N)
    R, neff = sd_all.finish()
    # n = 14 samples per split half: the reference's R-hat mixes W = mean of stds (Q8) with B, so
    # stationary chains sit near sqrt((n-1)/n + B/(n W)) ~ 1.04 here, the same in every dimension
    assert np.all(np.isfinite(R)) and np.all(np.abs(R - 1) < 0.1) and R.std() < 0.01
    assert np.all(neff > 0)
    cut = N // 2 + 40
    qa, ca, sa = run(0, cut)
    qb, cb, sb = run(cut, N)
    assert torch.equal(torch.cat([qa, qb]), q_all)
    assert ca[H.CNT_LEAPFROG] + cb[H.CNT_LEAPFROG] == c_all[H.CNT_LEAPFROG]
    assert ca[H.CNT_ACCEPT] + cb[H.CNT_ACCEPT] == c_all[H.CNT_ACCEPT]
    for k in ("shift", "s1", "s2"):
        assert torch.equal(torch.cat([getattr(sa, k), getattr(sb, k)]), getattr(sd_all, k))
    nl = sd_all.n - 1                      # lags t < n exist (rows past them are not variogram sums)
    torch.testing.assert_close(sa.vsum[:nl] + sb.vsum[:nl], sd_all.vsum[:nl], rtol=1e-12, atol=0)


@pytest.mark.parametrize("fp_mode", ["fast", "exact"])
def test_dense_production_kernel_vs_oracle(fp_mode):
    """BASELINE config 3's kernel (rho=0.95 dense precision, f64 MFMA gradient, L-ordered tiles,
    Philox) at 80 chains (5 tiles, so the per-iteration sort really permutes chains)."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    N, D, Niter, wu, seed = 80, 100, 12, 3, 0xC3
    cov = O.mvn_cov(D, 0.95)
    rs = np.random.RandomState(5)
    q_start = rs.standard_normal((N, D)) @ np.linalg.cholesky(cov).T
    h = HMC_sampler(D, None, None, Nchain=N, Niter=Niter, sampler_type="Random", L_low=5, L_high=20, dt=0.1,
                    warm_up_num=wu, target=MVNTarget(np.zeros(D), cov), rng="philox", seed=seed, fp_mode=fp_mode)
    h.gen_sample(q_start, verbose=False)
    p0, P = dense_momenta(seed, N, D, Niter)
    L, lnu = host_L_lnu(seed, np.arange(N, dtype=np.uint64), Niter, 5, 20)
    ref = O.gen_sample_random(O.HMCCore(FastMVN(np.zeros(D), cov), 0.1), q_start, N, Niter, wu, 1, 5, 20,
                              O.ReplayDraws(p0, P, L, lnu))
    assert h.accept_R == ref["accept_R"] and h.accept_R_warm_up == ref["accept_R_warm_up"]
    assert h.n_leapfrog == ref["n_leapfrog"]
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, 1:, 0], ref["E_chain"][:, 1:], rtol=1e-10)


class PhiloxNutsDraws(O.ReplayDraws):
    """The NUTS kernel's Philox streams as an oracle draw source: momenta per iteration and the
    k-th direction/uniform of an iteration from block (0x80000000 + k, iteration, chain)."""

    def __init__(self, seed, p0, P):
        super().__init__(p0, P)
        self.seed = seed
        self.it = {}
        self.k = {}

    def p(self, m, i):
        self.it[m], self.k[m] = i, 0
        return super().p(m, i)

    def _block(self, m):
        w = words(KDRAW + self.k[m], self.it[m], m, self.seed)
        self.k[m] += 1
        return w

    def direction(self, m):
        return int(self._block(m)[0] & np.uint64(1))

    def uniform(self, m):
        w = self._block(m)
        return float(u53(w[2], w[3]))


@pytest.mark.parametrize("fp_mode", ["fast", "exact"])
def test_nuts_production_kernel_vs_oracle(fp_mode):
    """BASELINE config 5's kernel (NUTS, rho=0.95, D=100, d_max=10, chain queue, Philox):
    32 chains x 6 iterations vs the oracle driven by the same Philox streams."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.target import MVNTarget
    N, D, Niter, wu, seed, d_max = 32, 100, 6, 2, 0xAB5, 10
    cov = O.mvn_cov(D, 0.95)
    rs = np.random.RandomState(9)
    q_start = rs.standard_normal((N, D)) @ np.linalg.cholesky(cov).T
    h = HMC_sampler(D, None, None, Nchain=N, Niter=Niter, warm_up_num=wu, sampler_type="NUTS", dt=0.1, d_max=d_max,
                    target=MVNTarget(np.zeros(D), cov), rng="philox", seed=seed, fp_mode=fp_mode)
    h.gen_sample_NUTS(q_start, 0, False, on_dmax="break")
    p0, P = dense_momenta(seed, N, D, Niter)
    ref = O.gen_sample_nuts(O.HMCCore(FastMVN(np.zeros(D), cov), 0.1), q_start, N, Niter, wu, 1, d_max,
                            PhiloxNutsDraws(seed, p0, P), on_dmax="break")
    assert h.n_leapfrog == ref["n_leapfrog"]
    assert h.n_unstable == ref["n_unstable"]
    np.testing.assert_allclose(h.q_chain, ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(h.E_chain[:, 1:, 0], ref["E_chain"][:, 1:], rtol=1e-10)


# ---------------------------------------------------------------- the benched sizes (properties)
def _stationary_start(N, D, rho, seed):
    cov = O.mvn_cov(D, rho)
    return cov, np.random.RandomState(seed).standard_normal((N, D)) @ np.linalg.cholesky(cov).T


def _law_checks(x, rho, N):
    """x (N, D) one draw per chain from N(0, Sigma): unit variances, corr(d0, d1) = rho."""
    assert np.abs(x.mean(axis=0)).max() < 6 / np.sqrt(N)
    assert np.abs(x.var(axis=0) - 1).max() < 6 * np.sqrt(2 / N)
    assert abs(np.corrcoef(x[:, 0], x[:, 1])[0, 1] - rho) < 6 * (1 - rho ** 2) / np.sqrt(N)


def test_dense_c3_scale_stationary_and_sharded():
    """BASELINE config 3 at its benched size (262,144 chains = 16,384 MFMA tiles, L-ordered):
    the stationary law N(0, Sigma) is preserved, and running the two halves as separate shards
    (chain_offset) gives bit-identical chains, so the per-iteration tile ordering over 16k tiles
    never changes a value."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, D, rho, Niter = 262144, 100, 0.95, 4
    cov, q_start = _stationary_start(N, D, rho, 21)
    qs = torch.as_tensor(q_start, device="cuda")

    def run(lo, hi):
        eng = RandomEngine(MVNTarget(np.zeros(D), cov), hi - lo, Niter, 1, 1, 5, 20, 0.1, rng="philox", seed=5,
                           fp_mode="fast", chain_offset=lo, store_chain=False)
        assert eng._order is not None
        eng.init(qs[lo:hi].contiguous())
        eng.run(1, Niter + 1)
        torch.cuda.synchronize()
        return eng.q.cpu().numpy(), eng.read_counters()

    q_all, c_all = run(0, N)
    _law_checks(q_all, rho, N)
    from hmc_amd import _lib as H
    acc = c_all[H.CNT_ACCEPT] / (N * Niter)
    assert 0.5 < acc < 1.0
    assert abs(c_all[H.CNT_LEAPFROG] / (N * Niter) - 12.0) < 0.05
    qa, ca = run(0, N // 2 + 40)          # ragged split: neither half is a whole number of tiles
    qb, cb = run(N // 2 + 40, N)
    assert np.array_equal(np.concatenate([qa, qb]), q_all)
    assert ca[H.CNT_LEAPFROG] + cb[H.CNT_LEAPFROG] == c_all[H.CNT_LEAPFROG]


def test_nuts_c5_scale_stationary_and_sharded():
    """BASELINE config 5 at its benched size (65,536 chains, chain queue over persistent waves):
    stationary law preserved, and every chain's result is independent of queue contention and
    sharding (two shards == one launch, bitwise; leapfrog counts add up)."""
    from hmc_amd.engine import NutsEngine
    from hmc_amd.target import MVNTarget
    from hmc_amd import _lib as H
    N, D, rho, Niter = 65536, 100, 0.95, 2
    cov, q_start = _stationary_start(N, D, rho, 22)
    qs = torch.as_tensor(q_start, device="cuda")

    def run(lo, hi):
        eng = NutsEngine(MVNTarget(np.zeros(D), cov), hi - lo, Niter, 1, 1, 10, 0.1, rng="philox", seed=6,
                         fp_mode="fast", chain_offset=lo, store_chain=False, on_dmax="break")
        eng.init(qs[lo:hi].contiguous())
        eng.run(1, Niter + 1)
        torch.cuda.synchronize()
        return eng.q.cpu().numpy(), eng.read_counters()

    q_all, c_all = run(0, N)
    _law_checks(q_all, rho, N)
    lf_per_it = c_all[H.CNT_LEAPFROG] / (N * Niter)
    assert 100 < lf_per_it < 600                       # observed mean ~245 at c5
    assert c_all[H.CNT_DMAX] < 0.01 * N * Niter
    qa, ca = run(0, 20000)
    qb, cb = run(20000, N)
    assert np.array_equal(np.concatenate([qa, qb]), q_all)
    assert ca[H.CNT_LEAPFROG] + cb[H.CNT_LEAPFROG] == c_all[H.CNT_LEAPFROG]
