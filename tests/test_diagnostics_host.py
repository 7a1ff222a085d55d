"""Host half of the diagnostics, no GPU: the vectorised ESS termination (hmc_amd.diagnostics.
ess_vectorised, all dimensions at once) against the oracle's per-dimension restatement of
utils.py:130-157 (oracle.hmc_oracle.ess_from_variogram), including the Q9 early exit, NaN
variances, runs that never stop and short chains."""
import numpy as np
import pytest

from oracle import hmc_oracle as O
from hmc_amd.diagnostics import ess_vectorised


@pytest.mark.parametrize("seed", range(6))
def test_ess_vectorised_matches_oracle_loop(seed):
    rs = np.random.RandomState(seed)
    for _ in range(200):
        n = int(rs.randint(3, 80))
        m = 2 * int(rs.randint(2, 50))
        D = 9
        var = rs.uniform(0.2, 3.0, D)
        a = rs.uniform(-0.5, 0.995, D)
        lags = np.arange(1, n)[:, None]
        rho = a[None, :] ** lags + rs.normal(0, rs.choice([1e-3, 0.05]), (n - 1, D))
        rho[:, 0] = 0.005                              # Q9: rho_1 < 0.01 -> sum 0
        if rs.rand() < 0.2:
            var[1] = 0.0                               # 0/0 -> NaN path
        Vt = (1 - rho) * 2 * var[None, :]
        ne, need = ess_vectorised(Vt, var, n, m, complete=True)
        assert not need.any()
        for d in range(D):
            with np.errstate(all="ignore"):
                ref, t_needed = O.ess_from_variogram(var[d], list(Vt[:, d]), n, m)
            assert (np.isnan(ref) and np.isnan(ne[d])) or ne[d] == pytest.approx(ref, rel=1e-13), (n, d)
            # with only the lags the reference read, the answer is already final
            T = max(2, min(n - 1, t_needed))
            ne2, need2 = ess_vectorised(Vt[:T, d:d + 1], var[d:d + 1], n, m, complete=T >= n - 1)
            if not need2[0]:
                assert (np.isnan(ref) and np.isnan(ne2[0])) or ne2[0] == pytest.approx(ref, rel=1e-13)


def test_ess_vectorised_flags_missing_lags():
    n, m = 60, 10
    var = np.ones(2)
    rho = np.full((10, 2), 0.5)                        # never turns negative within 10 lags
    Vt = (1 - rho) * 2
    ne, need = ess_vectorised(Vt, var, n, m, complete=False)
    assert need.all() and np.isnan(ne).all()
    ne, need = ess_vectorised(Vt, var, n, m, complete=False, truncate=True)   # streaming: sum ends at T
    assert not need.any()
    assert ne == pytest.approx(m * n / (1 + 2 * 0.5 * 9))
