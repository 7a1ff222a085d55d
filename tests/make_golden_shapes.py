"""Input shapes shared by tests and tests/golden/make_golden.py (data only, no reference code)."""
import numpy as np


def dense_cov_p(D):
    """A full (non-diagonal) SPD mass matrix for the Q3 cov_p case (samplers.py:352-356)."""
    i = np.arange(D)
    return 0.5 * np.exp(-np.abs(i[:, None] - i[None, :]) / 3.0) + np.diag(np.linspace(0.6, 1.4, D))
