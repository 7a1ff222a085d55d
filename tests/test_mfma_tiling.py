"""Host check of the matrix-core lag pass's tiling (csrc/hmc_diag.hip k_conv_mfma / k_mfma_dims):
the loops of the kernel restated in NumPy, for every n the pass takes (96 .. 208).

The kernel adds, for anchor step bi (b = 16 bi + 15), tile ti (T = 16 (ti - 1)) with
ti <= tl(bi) = v + 1 - bi (v = (n - 1) // 16), and MFMA entry (t', s):
    acc[ti][t'][s] += sum_k y_k[b + T + t'] * y_k[b - s]     (lag L = T + t' + s, anchor b - s)
over rows padded with zeros outside [0, n); k_mfma_dims then reads lag t = 16 q + r as
    C_t = sum_{s<=r} acc[q+1][r-s][s] + sum_{s>r} acc[q][r+16-s][s].
Checked here: every product y_i y_{i+L} with 0 <= i, i + L < n, L >= 1 is added exactly once, every
row the loops read lies in the LDS series [-16, n + 29], the MFMA count of c3's n = 200 is 104 per
chain group, and C_t from the emulated accumulators equals the direct sum."""
import numpy as np
import pytest


def _steps(n):
    v = (n - 1) // 16
    for bi in range(v + 1):
        for ti in range(v + 2 - bi):            # ti <= tl = v + 1 - bi (and <= NT - 1 = v + 1)
            yield bi, ti


@pytest.mark.parametrize("n", [96, 99, 128, 130, 150, 177, 199, 200, 208])
def test_each_lag_product_once(n):
    count = {}
    rows = []
    for bi, ti in _steps(n):
        b, T = 16 * bi + 15, 16 * (ti - 1)
        for tp in range(16):
            for s in range(16):
                i, L = b - s, T + tp + s
                rows += [b + T + tp, b - s]
                if L >= 1 and i >= 0 and i + L < n:
                    count[(i, L)] = count.get((i, L), 0) + 1
    want = {(i, L) for L in range(1, n) for i in range(n - L)}
    assert set(count) == want
    assert set(count.values()) == {1}
    assert min(rows) >= -16 and max(rows) <= n + 29     # inside the zero-padded LDS series


def test_mfma_count_c3():
    assert sum(1 for _ in _steps(200)) == 104
    assert sum(1 for _ in _steps(99)) == 35


@pytest.mark.parametrize("n", [99, 200])
def test_emulated_accumulators_give_the_lag_sums(n):
    rs = np.random.RandomState(n)
    K = 4
    y = rs.standard_normal((K, n))
    pad = np.zeros((K, n + 64))
    pad[:, 16:16 + n] = y                       # row r at column 16 + r, zeros around

    def Y(r):
        return pad[:, 16 + r]
    v = (n - 1) // 16
    acc = np.zeros((v + 2, 16, 16))
    for bi, ti in _steps(n):
        b, T = 16 * bi + 15, 16 * (ti - 1)
        A = np.stack([Y(b + T + tp) for tp in range(16)])   # [t'][k]
        B = np.stack([Y(b - s) for s in range(16)], axis=1)  # [k][s]
        acc[ti] += A @ B
    for t in range(1, n):
        q, r = divmod(t, 16)
        c = sum(acc[q + 1][r - s][s] for s in range(r + 1)) + sum(acc[q][r + 16 - s][s] for s in range(r + 1, 16))
        direct = float((y[:, t:] * y[:, :n - t]).sum())
        assert abs(c - direct) <= 1e-12 * max(1.0, abs(direct)) + 1e-12
