"""hmc_convergence_sums (the one-pass R-hat / variogram sums behind convergence_stats,
utils.py:77-179) against a float64 NumPy restatement of the same sums, over the shapes both
lag kernels meet: the direct-to-LDS kernel (even D, 16-B aligned rows) and the register-staged
one (odd D, odd strides, a misaligned view), n below / at / above the chunk and lag widths, one
or few split chains per block group, and every lag width tmax in {8, 16, 32, 64}.

The sums are the ones include/hmc.h documents: rows [sum_j std_j, sum_j (mean_j - S),
sum_j (mean_j - S)^2, V_1 .. V_tmax, V_{n-1}] with S = the view's first sample and
V_t = sum_j sum_{s < n-t} (x_j[s+t] - x_j[s])^2 (0 for t >= n)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expected(view, n, tmax):
    """view: (Nchain, >= 2n, D) float64 NumPy; split chain 2m+h = view[m, h n : (h+1) n]."""
    N, _, D = view.shape
    xs = np.concatenate([view[:, :n], view[:, n:2 * n]], axis=0)      # (2N, n, D)
    S = view[0, 0]
    mean = xs.mean(axis=1)
    std = xs.std(axis=1, ddof=1)
    out = np.zeros((4 + tmax, D))
    out[0] = std.sum(axis=0)
    out[1] = (mean - S).sum(axis=0)
    out[2] = ((mean - S) ** 2).sum(axis=0)
    for t in range(1, min(tmax, n - 1) + 1):
        out[2 + t] = ((xs[:, t:] - xs[:, :-t]) ** 2).sum(axis=(0, 1))
    if n >= 2:
        out[3 + tmax] = ((xs[:, n - 1] - xs[:, 0]) ** 2).sum(axis=0)      # lag n - 1
    return out


CASES = [
    # (Nchain, Niter, Dtot, dim slice start, thin, warm-up, tmax)
    (37, 201, 100, 0, 1, 1, 64),       # LDS kernel: headline D, n = 100
    (5, 41, 100, 0, 1, 1, 16),         # n = 20: one full chunk + a ragged one
    (3, 9, 64, 0, 1, 1, 8),            # n = 4 < TW
    (64, 67, 130, 0, 1, 3, 32),        # n = 32 = T; 3 dim tiles, a ragged last one
    (2, 260, 2, 0, 1, 0, 64),          # D = 2: one dim pair; n = 130 > tmax
    (1000, 34, 100, 0, 1, 0, 16),      # many split chains per block group, n = 17
    (9, 300, 101, 0, 3, 2, 64),        # odd D -> register-staged kernel, thinned view
    (9, 300, 101, 1, 1, 1, 64),        # D = 100 view, odd row stride -> register-staged kernel
    (9, 300, 100, -1, 1, 1, 64),       # even strides, storage at an 8-B offset -> register-staged
    (11, 120, 100, 0, 3, 0, 32),       # even stride x thin: LDS kernel on a thinned view
    (7, 101, 100, 0, 1, 1, 48),        # n = 50 (the bench window), 48 lags: 3-wave blocks
    (4, 201, 130, 0, 1, 1, 48),        # n = 100 > 48
    (6, 101, 101, 0, 1, 1, 48),        # odd D, 48 lags -> register-staged kernel (an idle wave)
    # complete passes (tmax >= n - 2): lag groups up to n - 1 - tail, the tail in difference form
    (6, 199, 100, 0, 1, 1, 97),        # n = 99 (c4's halves): two groups of 48 + a tail of 2
    (3, 401, 100, 0, 1, 1, 198),       # n = 200 (c3's window): four groups + a tail of 7
    (5, 115, 70, 0, 1, 1, 55),         # n = 57: one group + the longest tail, 8
    (5, 117, 70, 0, 1, 1, 56),         # n = 58: two groups (a tail of 9 would exceed 8)
    (4, 240, 100, 0, 1, 1, 150),       # tmax beyond n - 1 = 119: the lags past it are 0
    # complete passes of 96 <= n <= 208 take the matrix cores (k_conv_mfma, Hankel tiles;
    # hmc_diag.hip kMfmaMinN / kMfmaMaxN)
    (3, 193, 13, 0, 1, 1, 94),         # n = 96 (the smallest), D = 13: a partial dim group; 6 split
                                       # chains: one full chain group of 4 and a ragged one
    (3, 257, 13, 0, 1, 1, 126),        # n = 128, the same groups
    # the static-triangle instances of 97 <= n <= 111 (k_conv_mfma<8, E4, 6>): each anchor step's
    # last tile as E4 = 1, 2, 3 4x4x4 MFMAs (n % 16 = 1, 5, 9), whole (n % 16 = 14); n = 112 runtime
    (3, 195, 13, 0, 1, 1, 95),         # n = 97, E4 = 1
    (5, 203, 21, 0, 1, 1, 99),         # n = 101, E4 = 2, a partial dim group, a ragged chain group
    (3, 211, 13, 0, 1, 1, 103),        # n = 105, E4 = 3
    (6, 221, 17, 0, 1, 1, 108),        # n = 110, static triangle, whole last tiles
    (3, 225, 13, 0, 1, 1, 110),        # n = 112 (16 | n): the runtime-bound instance
    # k_conv_mfma<14, E4, 12> (193 <= n <= 207): E4 = 1, 2, 3 (c3's n = 200), whole last tiles
    (3, 387, 13, 0, 1, 1, 191),        # n = 193, E4 = 1
    (5, 395, 21, 0, 1, 1, 195),        # n = 197, E4 = 2, a partial dim group, a ragged chain group
    (3, 401, 13, 0, 1, 1, 198),        # n = 200, E4 = 3
    (3, 413, 13, 0, 1, 1, 204),        # n = 206, static triangle, whole last tiles
    (2, 417, 100, 0, 1, 1, 206),       # n = 208 (the largest): every tile and anchor step
    (2, 481, 100, 0, 1, 1, 238),       # n = 240: past the matrix-core range (VALU lag kernel)
    (5, 300, 101, 1, 1, 1, 200),       # n = 149, a D = 100 view with odd row stride; tmax beyond n - 1
    (4, 452, 9, -1, 1, 0, 224),        # storage at an 8-B offset, n = 226, odd D
    (7, 301, 64, 0, 1, 1, 148),        # n = 150, D = 64: full dim groups
    (5, 1200, 24, 0, 3, 3, 197),       # thinned view (every 3rd row), n = 199
]


@pytest.mark.parametrize("N,Niter,Dtot,d0,thin,wu,tmax", CASES)
def test_convergence_sums_vs_numpy(N, Niter, Dtot, d0, thin, wu, tmax):
    from hmc_amd.diagnostics import _Split, convergence_sums

    rng = np.random.default_rng(N * 1000 + Niter + Dtot + tmax)
    # AR(1) chains around a per-dim offset, so that lags carry structure and shifts matter
    q = np.empty((N, Niter, Dtot))
    q[:, 0] = rng.normal(size=(N, Dtot))
    for t in range(1, Niter):
        q[:, t] = 0.8 * q[:, t - 1] + rng.normal(size=(N, Dtot))
    q += rng.normal(size=Dtot) * 5.0
    if d0 >= 0:
        t_dev = torch.as_tensor(q).cuda()[:, :, d0:]
    else:                              # the same array one double into its storage (8-B aligned only)
        flat = torch.zeros(q.size + 1, dtype=torch.float64, device="cuda")
        flat[1:] = torch.as_tensor(q.reshape(-1)).cuda()
        t_dev = flat[1:].view(q.shape)
        assert t_dev.data_ptr() % 16 == 8
        d0 = 0
    sp = _Split(t_dev, thin, wu)
    got = convergence_sums(sp, tmax).cpu().numpy()
    view = q[:, wu::thin, d0:]
    want = _expected(view, sp.n, tmax)
    np.testing.assert_allclose(got, want, rtol=1e-10, atol=1e-9 * np.abs(want).max())


@pytest.mark.parametrize("d0,d1,wu", [(3, 50, 0), (1, 101, 4), (0, 7, 2)])
def test_convergence_stats_dim_sliced_view_vs_oracle(d0, d1, wu):
    """convergence_stats on a non-contiguous, dim-sliced device view (q[:, 1:, d0:d1], row stride
    != D): the shift S must be the view's own first sample, not a position in a flattened copy
    (advisor r03).  R-hat and ESS equal the oracle's on the same NumPy slice."""
    from hmc_amd import diagnostics as G
    from oracle import hmc_oracle as O
    rs = np.random.RandomState(11 + d0)
    N, L, Dt = 16, 81, 101
    x = np.empty((N, L, Dt))
    x[:, 0] = rs.standard_normal((N, Dt))
    for t in range(1, L):
        x[:, t] = 0.6 * x[:, t - 1] + rs.standard_normal((N, Dt))
    x += np.linspace(-30.0, 30.0, Dt)                  # per-dim offsets: a wrong shift shows
    dev = torch.as_tensor(x).cuda()[:, 1:, d0:d1]
    assert not dev.is_contiguous()
    R, neff = G.convergence_stats(dev, thin_rate=1, warm_up_num=wu)
    R_ref, neff_ref = O.convergence_stats(x[:, 1:, d0:d1], thin_rate=1, warm_up_num=wu)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)


@pytest.mark.parametrize("D", [100, 7])
def test_convergence_stats_n50_vs_oracle(D):
    """Split chains of n = 50 (the bench window): the one pass takes lags 1..48 (conv_tmax) and
    lag 49 (its extra row), so the dimensions whose ESS criterion reaches its final check (slow
    mixing) need no further pass.  R-hat and ESS equal the oracle's (utils.py:77-179 restated)."""
    from hmc_amd import diagnostics as G
    from oracle import hmc_oracle as O
    rs = np.random.RandomState(5)
    N, L = 24, 101
    rho = np.linspace(0.0, 0.995, D)
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D)) - 2.0
    for t in range(1, L):
        x[:, t] = -2.0 + rho * (x[:, t - 1] + 2.0) + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    R, neff = G.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    assert G.LAST_INFO["tmax"] == 48 and G.LAST_INFO["lags"] == 49 and G.LAST_INFO["fallback_dims"] == 0
    R_ref, neff_ref = O.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)


@pytest.mark.parametrize("D", [20, 7])
def test_convergence_stats_mfma_window_vs_oracle(D):
    """c3's window shape (split chains of n = 200, every lag 1..199 in one pass on the matrix cores)
    on slowly to fast mixing AR(1) dims: R-hat and ESS equal the oracle's convergence_stats
    (utils.py:77-179 restated), no fallback pass."""
    from hmc_amd import diagnostics as G
    from oracle import hmc_oracle as O
    rs = np.random.RandomState(7 + D)
    N, L = 10, 401
    rho = np.linspace(0.0, 0.995, D)
    x = np.empty((N, L, D))
    x[:, 0] = rs.standard_normal((N, D)) + 1.5
    for t in range(1, L):
        x[:, t] = 1.5 + rho * (x[:, t - 1] - 1.5) + np.sqrt(1 - rho * rho) * rs.standard_normal((N, D))
    R, neff = G.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    assert G.LAST_INFO["tmax"] == 198 and G.LAST_INFO["lags"] == 199 and G.LAST_INFO["fallback_passes"] == 0
    R_ref, neff_ref = O.convergence_stats(x[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-10)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)


@pytest.mark.parametrize("n,slope", [(99, 1e3), (200, 1e3), (128, 1e5)])
def test_mfma_trending_halves_vs_numpy(n, slope):
    """Complete passes on the matrix cores (96 <= n <= 208) use V_t = sum sq + sum sq - 2 C_t, an
    expanded form that cancels when the samples drift far from the series' first sample (advisor
    r05): strongly trending split halves, x = slope * t + noise.  The sums still equal a float64
    NumPy restatement of the difference form to the suite's tolerance, and R-hat / ESS equal the
    oracle's convergence_stats (utils.py:77-179)."""
    from hmc_amd.diagnostics import _Split, convergence_stats, convergence_sums
    from oracle import hmc_oracle as O
    rs = np.random.default_rng(n)
    N, D = 12, 9
    rows = 2 * n + 1
    t = np.arange(rows, dtype=np.float64)
    q = slope * t[None, :, None] * np.linspace(0.5, 1.5, D)[None, None, :] + rs.normal(size=(N, rows, D))
    dev = torch.as_tensor(q).cuda()
    sp = _Split(dev, 1, 1)
    assert sp.n == n
    got = convergence_sums(sp, n - 2).cpu().numpy()
    want = _expected(q[:, 1:], n, n - 2)
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12 * np.abs(want).max())
    R, neff = convergence_stats(dev[:, 1:, :], thin_rate=1, warm_up_num=0)
    R_ref, neff_ref = O.convergence_stats(q[:, 1:, :], thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R, R_ref, rtol=1e-9)
    np.testing.assert_allclose(neff, neff_ref, rtol=1e-8)
