"""Every lag of the reference's ESS loop (utils.py:128-157) without a stored q_chain, and on
stored windows of any length.

* hmc_half_sums: the one-read lag kernel over ONE split half per chain read in place from a
  circular streaming window (rows wrap), against a float64 NumPy restatement of the sums.
* StreamingDiagnostics in exact mode (RandomEngine.run_streaming feeding each half once complete):
  R-hat AND n_eff equal the oracle's convergence_stats (oracle/hmc_oracle.py, utils.py:77-179
  restated) in every dimension, including the slow-mixing ones whose loop runs to lag n - 1, at
  the c4 shape ratio (D = 1000, 200 samples: halves of 99) -- the VERDICT r04 item the bench's
  `truncated_dims: 0` rests on.
* Stored windows: a complete single pass for n = 200 (no fallback read), the fallback beyond 4096
  lags (n > 4193, advisor r04), and the dimension-sliced path for views whose chains exceed the lag
  kernel's 1 GiB offsets.
Tolerance: 1e-10 rel for R-hat (sums in another order), 1e-8 for n_eff (a ratio of such sums)."""
import numpy as np
import pytest
import torch

from oracle import hmc_oracle as O

pytestmark = pytest.mark.gpu


def _half_expected(x, tmax):
    """x: (N, n, D) one series per chain; rows of hmc_half_sums' output."""
    N, n, D = x.shape
    S = x[0, 0]
    mean = x.mean(axis=1)
    std = x.std(axis=1, ddof=1)
    out = np.zeros((4 + tmax, D))
    out[0] = std.sum(axis=0)
    out[1] = (mean - S).sum(axis=0)
    out[2] = ((mean - S) ** 2).sum(axis=0)
    for t in range(1, min(tmax, n - 1) + 1):
        out[2 + t] = ((x[:, t:] - x[:, :-t]) ** 2).sum(axis=(0, 1))
    out[3 + tmax] = ((x[:, n - 1] - x[:, 0]) ** 2).sum(axis=0)
    return out


@pytest.mark.parametrize("N,n,D,W,slot0", [(7, 99, 100, 121, 50),    # wraps after 71 samples
                                           (3, 200, 70, 240, 239),   # wraps after one sample
                                           (40, 17, 1000, 30, 0),    # no wrap, D = 1000
                                           (5, 57, 33, 57, 20),      # the half fills the window
                                           (9, 4, 64, 8, 6),         # tiny half
                                           # halves of 128 .. 208 that do not wrap: the matrix cores
                                           (6, 199, 100, 420, 201),  # c4 at 400 samples: the second half
                                           (3, 130, 13, 131, 0),     # D = 13, three series (< one group)
                                           (9, 208, 40, 208, 0)])    # the largest, the window exactly
def test_half_sums_circular_window_vs_numpy(N, n, D, W, slot0):
    from hmc_amd import _lib as H
    rng = np.random.default_rng(N + n + D + W)
    x = np.empty((N, n, D))
    x[:, 0] = rng.normal(size=(N, D))
    for t in range(1, n):
        x[:, t] = 0.9 * x[:, t - 1] + rng.normal(size=(N, D))
    x += rng.normal(size=D) * 4.0
    win = rng.normal(size=(N, W, D)) * 1e6                  # rows outside the half: garbage
    for s in range(n):
        win[:, (slot0 + s) % W] = x[:, s]
    wt = torch.as_tensor(win).cuda()
    tmax = max(1, n - 2)
    L = H.lib()
    work = torch.zeros(L.hmc_convergence_work_size(N, D, tmax), dtype=torch.float64, device="cuda")
    out = torch.zeros((4 + tmax, D), dtype=torch.float64, device="cuda")
    H.check(L.hmc_half_sums(wt.data_ptr(), N, wt.stride(0), wt.stride(1), D, W, slot0, n, tmax, H.ptr(work),
                            H.ptr(out), torch.cuda.current_stream().cuda_stream), "hmc_half_sums")
    want = _half_expected(x, tmax)
    np.testing.assert_allclose(out.cpu().numpy(), want, rtol=1e-10, atol=1e-9 * np.abs(want).max())


def test_half_sums_rejects_bad_window():
    from hmc_amd import _lib as H
    L = H.lib()
    wt = torch.zeros((2, 10, 4), dtype=torch.float64, device="cuda")
    work = torch.zeros(1 << 16, dtype=torch.float64, device="cuda")
    out = torch.zeros((64, 4), dtype=torch.float64, device="cuda")
    for W, slot0, n in ((10, 10, 5), (10, 0, 11), (-1, 0, 5)):
        with pytest.raises(AssertionError):
            H.check(L.hmc_half_sums(wt.data_ptr(), 2, 40, 4, 4, W, slot0, n, 3, H.ptr(work), H.ptr(out), None), "x")


def _engine_pair(D, N, Niter, wu, thin, seed):
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    tgt = MVNTarget(np.zeros(D), np.eye(D))
    q0 = torch.as_tensor(np.random.RandomState(seed).standard_normal((N, D)) * 1.5).cuda()

    def engine(store):
        e = RandomEngine(tgt, N, Niter, wu, thin, 5, 20, 0.1, rng="philox", seed=seed, fp_mode="fast",
                         store_chain=store)
        e.init(q0)
        return e
    return engine


@pytest.mark.parametrize("D,N,Niter,wu,thin,step,feed,per_step", [
    (1000, 16, 240, 41, 1, 20, 200, True),  # c4's shape ratio: 200 rows, halves of 99 (the bench's calls)
    (100, 64, 150, 10, 1, 16, 80, False),   # a window of one half: the second half wraps
    (60, 40, 200, 5, 3, 8, 200, False),     # thinned rows
])
def test_streaming_exact_matches_oracle_every_dim(D, N, Niter, wu, thin, step, feed, per_step):
    from hmc_amd.diagnostics import LAST_INFO, StreamingDiagnostics
    make = _engine_pair(D, N, Niter, wu, thin, seed=D + N)
    full = make(True)
    full.run(1, Niter + 1)
    qc = full.q_chain[:, 1:, :].cpu().numpy()
    st = make(False)
    sd = StreamingDiagnostics(N, D, st.L_chain - 1, tmax=16)
    feed = step * (feed // step)
    if per_step:
        for a in range(1, Niter + 1, step):
            st.run_streaming(sd, a, min(a + step, Niter + 1), step, feed=feed)
    else:
        st.run_streaming(sd, 1, Niter + 1, step, feed=feed)
    assert sd.mode == "exact"
    W = st._stream[1].shape[1]
    # both halves whole when that fits the segment mode's window, else one half + a launch's rows
    W_seg = 16 + (feed + step) // thin + 2
    W2 = 2 * sd.n + -(-step // thin) + 2
    assert W == (W2 if W2 <= W_seg else sd.n + -(-step // thin) + 2)
    assert (W < W2) == (feed == 80)
    R, neff = sd.finish()
    assert sd.info["truncated_dims"] == 0 and LAST_INFO["mode"] == "streaming-exact"
    assert torch.equal(st.q, full.q)
    R_ref, neff_ref = O.convergence_stats(qc, thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)          # EVERY dimension


def test_streaming_exact_checkpoint_resume(tmp_path):
    """Checkpoint between the two halves (exact mode), resume in a fresh engine: identical."""
    from hmc_amd.diagnostics import StreamingDiagnostics
    make = _engine_pair(100, 128, 160, 20, 1, seed=3)

    def diag(e):
        return StreamingDiagnostics(e.N, e.D, e.L_chain - 1, tmax=16)
    ref = make(False)
    sref = diag(ref)
    ref.run_streaming(sref, 1, 161, 10, feed=80)
    R_ref, neff_ref = sref.finish()
    a = make(False)
    sa = diag(a)
    a.run_streaming(sa, 1, 121, 10, feed=80)                  # half 0 (rows 1..70) fed, half 1 open
    assert sa.halves == [0]
    path = str(tmp_path / "c.npz")
    a.save(path, 121, diag=sa)
    b = make(False)
    sb = diag(b)
    assert b.restore(path, diag=sb) == 121
    b.run_streaming(sb, 121, 161, 10, feed=80)
    R, neff = sb.finish()
    np.testing.assert_array_equal(R, R_ref)
    np.testing.assert_array_equal(neff, neff_ref)


def test_streaming_checkpoint_inside_first_half(tmp_path):
    """Checkpoint INSIDE split half 0 (exact mode chosen, nothing fed yet: diag.pos = 0, the open
    half only in the window).  The checkpoint carries the mode and the window size (advisor r05): a
    resume with another feed keeps exact mode and, when the window size is unchanged, matches the
    uninterrupted run bit for bit; one whose feed asks for another window size is refused instead of
    summing half 0 from a zeroed window."""
    from hmc_amd.diagnostics import StreamingDiagnostics
    make = _engine_pair(100, 128, 160, 20, 1, seed=5)

    def diag(e):
        return StreamingDiagnostics(e.N, e.D, e.L_chain - 1, tmax=16)
    ref = make(False)
    sref = diag(ref)
    ref.run_streaming(sref, 1, 161, 10, feed=80)
    R_ref, neff_ref = sref.finish()
    a = make(False)
    sa = diag(a)
    a.run_streaming(sa, 1, 41, 10, feed=80)                   # rows 1..20 of half 0 (70 rows)
    assert sa.pos == 0 and sa.halves == [] and sa.mode == "exact"
    path = str(tmp_path / "c.npz")
    a.save(path, 41, diag=sa)
    # feed 20 alone would choose segment mode (n = 70 > tmax + 20); the recorded mode wins, and the
    # window is the same 82 rows (one half + a launch of 10 rows + 2)
    b = make(False)
    sb = diag(b)
    assert b.restore(path, diag=sb) == 41 and sb.mode == "exact" and sb.window_rows == 82
    b.run_streaming(sb, 41, 161, 10, feed=20)
    R, neff = sb.finish()
    np.testing.assert_array_equal(R, R_ref)
    np.testing.assert_array_equal(neff, neff_ref)
    # feed 160 would hold both halves (152 rows): refused, the open half is not dropped
    c = make(False)
    sc = diag(c)
    assert c.restore(path, diag=sc) == 41
    with pytest.raises(AssertionError, match="window"):
        c.run_streaming(sc, 41, 161, 10, feed=160)


def test_convergence_stats_n200_one_pass():
    """c3's window shape (n = 200, slow mixing in every dim): one complete pass, no fallback."""
    from hmc_amd import diagnostics as G
    rs = np.random.RandomState(8)
    N, L, D = 12, 401, 9
    rho = np.linspace(0.9, 0.995, D)
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D))
    for t in range(1, L):
        x[:, t] = rho * x[:, t - 1] + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    R, neff = G.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    assert G.LAST_INFO["fallback_passes"] == 0 and G.LAST_INFO["lags"] == 199
    R_ref, neff_ref = O.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)


def test_convergence_stats_fallback_beyond_4096_lags():
    """n = 4300 > 4193 with a slow-mixing dimension: the fallback reads lags 97 .. 4299 in one pass
    (advisor r04: these were refused above 4096 lags)."""
    from hmc_amd import diagnostics as G
    rs = np.random.RandomState(4)
    N, L, D = 3, 8601, 2
    rho = np.array([0.1, 0.9995])
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D))
    for t in range(1, L):
        x[:, t] = rho * x[:, t - 1] + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    R, neff = G.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    assert G.LAST_INFO["fallback_passes"] == 1 and G.LAST_INFO["lags"] > 4096 + 96
    R_ref, neff_ref = O.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)


def test_convergence_stats_dim_sliced_when_view_too_long(monkeypatch):
    """Views whose chains exceed the lag kernel's 1 GiB offsets go through contiguous dimension
    slices (forced here by a smaller bound): same R-hat and n_eff as one pass."""
    from hmc_amd import diagnostics as G
    rs = np.random.RandomState(2)
    N, L, D = 8, 161, 37
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D))
    for t in range(1, L):
        x[:, t] = 0.7 * x[:, t - 1] + rs.standard_normal((N, D))
    R0, n0 = G.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    real = G._fits
    monkeypatch.setattr(G, "_fits", lambda cs, ss, n, D_: real(cs, ss, n, D_) and D_ <= 10)
    R1, n1 = G.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    assert G.LAST_INFO["slices"] == 4
    np.testing.assert_allclose(R1, R0, rtol=1e-12)
    np.testing.assert_allclose(n1, n0, rtol=1e-10)
