"""Streaming diagnostics: R-hat / ESS of q_chain[:, 1:, :] from windows,
without storing q_chain.  Checked against the oracle's convergence_stats (utils.py:77-159
restated) on the same samples: R-hat exact to round-off; ESS identical for every dimension
whose reference termination criterion reads no lag beyond tmax (elsewhere the streaming sum
stops at tmax by design).  Tolerance: 1e-10 rel (fp64 sums in another order)."""
import numpy as np
import pytest
import torch

from oracle import hmc_oracle as O

pytestmark = pytest.mark.gpu


def _ar1(N, L, D, rho, seed):
    rs = np.random.RandomState(seed)
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D)) + 3.0
    for t in range(1, L):
        x[:, t] = 3.0 + rho * (x[:, t - 1] - 3.0) + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    return x


@pytest.mark.parametrize("tmax,seg", [(8, 7), (16, 1), (32, 50), (16, 200)])
def test_windows_match_oracle(tmax, seg):
    from hmc_amd.diagnostics import StreamingDiagnostics
    N, L, D = 37, 202, 70                                     # odd sample count: last sample unused
    q = _ar1(N, L, D, 0.4, seed=tmax + seg)
    R_ref, neff_ref = O.convergence_stats(q[:, 1:, :], thin_rate=1, warm_up_num=0)
    x = torch.as_tensor(q[:, 1:, :]).cuda()
    sd = StreamingDiagnostics(N, D, L - 1, tmax=tmax)
    p = 0
    while p < L - 1:
        rows = min(seg, L - 1 - p)
        carry = min(tmax, p)
        sd.update(x[:, p - carry:p + rows, :], carry, rows)   # strided view: no copy
        p += rows
    R, neff = sd.finish()
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    # ESS: identical wherever the reference's criterion needed no lag beyond tmax
    need = _lags_needed(q[:, 1:, :])
    ok = need <= tmax
    assert ok.sum() >= 5, (need, tmax)
    np.testing.assert_allclose(neff[ok], neff_ref[ok], rtol=1e-10)


@pytest.mark.parametrize("rho,tmax", [(0.97, 16), (0.6, 16), (0.9, 32)])
def test_truncated_dims_count_matches_oracle_loop(rho, tmax):
    """Slow-mixing chains: StreamingDiagnostics.finish() reports how many dimensions' reference
    ESS loop (utils.py:139-152) reads a lag beyond tmax -- exactly the dims whose streamed n_eff is
    a truncated sum -- and every other dim's n_eff equals the oracle's."""
    from hmc_amd.diagnostics import LAST_INFO, StreamingDiagnostics
    N, L = 24, 402
    D = 40
    rs = np.random.RandomState(int(rho * 100) + tmax)
    rhos = np.linspace(0.0, rho, D)                              # mixing from fast to slow per dim
    q = np.empty((N, L, D))
    q[:, 0] = rs.standard_normal((N, D))
    for t in range(1, L):
        q[:, t] = rhos * q[:, t - 1] + np.sqrt(1 - rhos * rhos) * rs.standard_normal((N, D))
    x = torch.as_tensor(q[:, 1:, :]).cuda()
    sd = StreamingDiagnostics(N, D, L - 1, tmax=tmax)
    p = 0
    while p < L - 1:
        rows = min(60, L - 1 - p)
        carry = min(tmax, p)
        sd.update(x[:, p - carry:p + rows, :], carry, rows)
        p += rows
    R, neff = sd.finish()
    need = _lags_needed(q[:, 1:, :])
    want = int((need > tmax).sum())
    assert sd.info["truncated_dims"] == want and LAST_INFO["truncated_dims"] == want
    if rho > 0.9:
        assert want > 0                                         # the case this report exists for
    _, neff_ref = O.convergence_stats(q[:, 1:, :], thin_rate=1, warm_up_num=0)
    ok = need <= tmax
    np.testing.assert_allclose(neff[ok], neff_ref[ok], rtol=1e-10)


def test_sampler_streaming_warns_on_truncation():
    """HMC_sampler(store_chain=False) with a tmax far below the chains' correlation time warns
    that its streamed n_eff is truncated (and by how many dims)."""
    from hmc_amd.samplers import HMC_sampler
    D, N = 6, 16
    tgt = O.MVNTarget(np.zeros(D), np.eye(D))
    h = HMC_sampler(D, tgt.V, tgt.dVdq, Nchain=N, Niter=400, sampler_type="Random", L_low=1, L_high=2,
                    dt=0.05, warm_up_num=0, store_chain=False, stream_tmax=8, iters_per_launch=20, rng="philox",
                    seed=3)
    h.gen_sample(np.full((N, D), 2.0), verbose=False)
    with pytest.warns(UserWarning, match="truncated"):
        h.compute_convergence_stats()
    assert h.stream_info["truncated_dims"] > 0


def _lags_needed(q):
    """Per dim, the largest variogram lag the reference's ESS loop reads (oracle restatement)."""
    chains, n = O.split_chains(q, thin_rate=1, warm_up_num=0)
    m = len(chains)
    W = np.mean(np.stack([np.std(c, ddof=1, axis=0) for c in chains]), axis=0)
    mw = np.stack([np.mean(c, axis=0) for c in chains])
    B = np.sum(np.square(mw - mw.mean(axis=0)), axis=0) * n / float(m - 1)
    var = W * (n - 1) / float(n) + B / float(n)
    D = q.shape[2]
    out = np.zeros(D, dtype=int)
    for i in range(D):
        Vt = [O.variogram(chains, i, t) for t in range(1, n)]
        out[i] = O.ess_from_variogram(var[i], Vt, n, m)[1]
    return out


@pytest.mark.parametrize("thin,wu,step,feed,per_step", [(1, 20, 10, 10, False), (3, 7, 16, 16, False),
                                                     (2, 0, 5, 5, False), (1, 20, 10, 40, True),
                                                     (3, 7, 8, 24, True)])
def test_engine_streaming_equals_stored_chain(thin, wu, step, feed, per_step):
    """Same Philox run twice: whole q_chain stored vs the sliding window feeding the
    streaming statistics."""
    from hmc_amd.diagnostics import StreamingDiagnostics, convergence_stats
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, D, Niter = 512, 100, 140
    tgt = MVNTarget(np.zeros(D), np.eye(D))
    q0 = torch.as_tensor(np.random.RandomState(1).standard_normal((N, D)) * 1.4).cuda()

    def engine(store):
        e = RandomEngine(tgt, N, Niter, wu, thin, 5, 20, 0.1, rng="philox", seed=9, fp_mode="fast",
                         store_chain=store)
        e.init(q0)
        return e
    full = engine(True)
    full.run(1, Niter + 1)
    R_ref, neff_ref = convergence_stats(full.q_chain[:, 1:, :], thin_rate=1, warm_up_num=0)
    st = engine(False)
    sd = StreamingDiagnostics(N, D, st.L_chain - 1, tmax=32)
    if per_step:   # bench.py's pattern: one call per launch, diagnostics fed every `feed` iterations
        for a in range(1, Niter + 1, step):
            st.run_streaming(sd, a, min(a + step, Niter + 1), step, feed=feed)
    else:
        st.run_streaming(sd, 1, Niter + 1, step, feed=feed)
    R, neff = sd.finish()
    assert torch.equal(st.q, full.q)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    ok = _lags_needed(full.q_chain[:, 1:, :].cpu().numpy()) <= 32
    assert ok.sum() >= 5
    np.testing.assert_allclose(neff[ok], neff_ref[ok], rtol=1e-10)


def test_checkpoint_resume_bitexact(tmp_path):
    """Checkpoint at iteration 60, resume in a fresh engine: identical to the uninterrupted
    run (Philox keyed by iteration), including the streaming statistics."""
    from hmc_amd.diagnostics import StreamingDiagnostics
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, D, Niter, wu = 256, 100, 120, 10
    tgt = MVNTarget(np.zeros(D), np.eye(D))
    q0 = torch.as_tensor(np.random.RandomState(2).standard_normal((N, D))).cuda()

    def make():
        e = RandomEngine(tgt, N, Niter, wu, 1, 5, 20, 0.1, rng="philox", seed=4, fp_mode="fast", store_chain=True)
        return e, StreamingDiagnostics(N, D, e.L_chain - 1, tmax=16)
    ref, sref = make()
    ref.init(q0)
    ref.run_streaming(sref, 1, Niter + 1, 10)
    R_ref, neff_ref = sref.finish()

    a, sa = make()
    a.init(q0)
    a.run_streaming(sa, 1, 61, 10)
    path = str(tmp_path / "ckpt.npz")
    a.save(path, 61, diag=sa)
    b, sb = make()
    it = b.restore(path, diag=sb)
    assert it == 61
    b.run_streaming(sb, it, Niter + 1, 10)
    R, neff = sb.finish()
    assert torch.equal(b.q, ref.q)
    assert torch.equal(b.E_chain, ref.E_chain)
    np.testing.assert_array_equal(b.read_counters(), ref.read_counters())
    np.testing.assert_array_equal(R, R_ref)
    np.testing.assert_array_equal(neff, neff_ref)


@pytest.mark.parametrize("sampler_type", ["Random", "NUTS"])
def test_sampler_streaming_mode_matches_oracle(sampler_type):
    """HMC_sampler(store_chain=False): the surface's streaming mode (samplers.py:53-64 ->
    utils.py:77-179 without a q_chain).  Replay-mode Random chains are bit-identical to the
    oracle's, so R-hat must equal the oracle's convergence_stats on the oracle's q_chain to
    1e-10 rel and ESS likewise wherever the reference reads no lag beyond stream_tmax."""
    from hmc_amd.samplers import HMC_sampler
    D, N, Niter, wu = 10, 24, 300, 60
    tgt = O.MVNTarget(np.zeros(D), np.eye(D))
    np.random.seed(77)
    q_start = O.start_pts(np.zeros(D), 2 * np.eye(D), N)
    if sampler_type == "Random":
        state = np.random.get_state()
        h = HMC_sampler(D, tgt.V, tgt.dVdq, Nchain=N, Niter=Niter, sampler_type="Random", L_low=5, L_high=20,
                        dt=0.1, warm_up_num=wu, store_chain=False, stream_tmax=48, iters_per_launch=16,
                        stream_feed=48)
        h.gen_sample(q_start, verbose=False)
        np.random.set_state(state)
        ref = O.gen_sample_random(O.HMCCore(tgt, 0.1), q_start, N, Niter, wu, 1, 5, 20, O.LiveDraws(D, np.eye(D)))
        qc = ref["q_chain"]
        np.testing.assert_allclose(h.E_chain[:, :, 0], ref["E_chain"], rtol=1e-12, atol=1e-12)   # as smoke()
    else:
        kw = dict(Nchain=N, Niter=Niter, sampler_type="NUTS", dt=0.2, warm_up_num=wu, rng="philox", seed=5,
                  fp_mode="fast", iters_per_launch=16)
        full = HMC_sampler(D, tgt.V, tgt.dVdq, **kw)
        full.gen_sample(q_start, verbose=False)
        qc = full.q_chain
        h = HMC_sampler(D, tgt.V, tgt.dVdq, store_chain=False, stream_tmax=48, stream_feed=48, **kw)
        h.gen_sample(q_start, verbose=False)
        assert np.array_equal(h.E_chain, full.E_chain)
    assert h.q_chain is None
    h.compute_convergence_stats()
    R_ref, neff_ref = O.convergence_stats(qc[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(h.R_q, R_ref, rtol=1e-10)
    ok = _lags_needed(qc[:, 1:, :]) <= 64          # stream_tmax 48 -> the 64-lag kernel
    assert ok.sum() >= 5
    np.testing.assert_allclose(h.n_eff_q[ok], neff_ref[ok], rtol=1e-10)


def test_checkpoint_rejects_other_engine(tmp_path):
    """A checkpoint restores only into an engine with the same dt, mass matrix and target."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    N, D = 64, 12
    mk = lambda dt, q0: RandomEngine(MVNTarget(q0, np.eye(D)), N, 20, 0, 1, 5, 20, dt, rng="philox",  # noqa: E731
                                     seed=1, fp_mode="fast")
    a = mk(0.1, np.zeros(D))
    a.init(torch.zeros((N, D), dtype=torch.float64).cuda())
    a.run(1, 5)
    path = str(tmp_path / "c.npz")
    a.save(path, 5)
    assert mk(0.1, np.zeros(D)).restore(path) == 5
    with pytest.raises(AssertionError, match="dt"):
        mk(0.2, np.zeros(D)).restore(path)
    with pytest.raises(AssertionError, match="target_sha256"):
        mk(0.1, np.full(D, 0.5)).restore(path)
