"""Multivariate-normal target descriptors for the GPU engine.

The reference hands the sampler two opaque Python closures, V(q) and dVdq(q)
(samplers.py:310-311, :327-328), built by every driver as
    V(q)    = -normal_lnL(q, q0, cov0)          (case1-script.py:39-43, utils.py:213-218)
    dVdq(q) = np.dot(inv_cov0, q - q0)          (case1-script.py:45-49)
The GPU cannot call Python closures, so the engine needs the MVN parameters
explicitly.  Two ways in:
  * `MVNTarget(q0, cov0)` passed as HMC_sampler(..., target=...);
  * `probe_closures(D, V, dVdq)`: affine probing of the closures
    (dVdq(0) and dVdq(e_i) give P = inv(cov0) column by column and q0; V(q0)
    gives the constant), verified at random points before it is trusted.
    For q0 = 0 (every reference driver) the probe is exact to the bit.
Targets that are not MVN are rejected (no CPU fallback exists in the product).
"""
import numpy as np


class MVNTarget:
    """q0 (D,), precision P = inv(cov0) (D, D), constant D*log(2*pi) + log det(cov0)."""

    def __init__(self, q0, cov0=None, prec=None, logdet_const=None):
        self.q0 = np.ascontiguousarray(q0, dtype=np.float64).reshape(-1)
        D = self.q0.size
        if prec is None:
            cov0 = np.asarray(cov0, dtype=np.float64)
            prec = np.linalg.inv(cov0)                     # case1-script.py:36
        self.prec = np.ascontiguousarray(prec, dtype=np.float64)
        if self.prec.shape != (D, D):
            raise AssertionError("precision must be (D, D)")
        if logdet_const is None:
            if cov0 is None:
                cov0 = np.linalg.inv(self.prec)
            # scipy's logpdf constant (utils.py:218): rank*log(2 pi) + log pseudo-det, via eigh
            w = np.linalg.eigvalsh(np.asarray(cov0, dtype=np.float64))
            logdet_const = D * np.log(2 * np.pi) + np.sum(np.log(w))
        self.logdet_const = float(logdet_const)
        off = self.prec - np.diag(np.diag(self.prec))
        self.diagonal = not np.any(off)
        self.identity = self.diagonal and np.all(np.diag(self.prec) == 1.0)
        self.zero_mean = not np.any(self.q0)

    @property
    def D(self):
        return self.q0.size

    def V(self, q):
        x = np.asarray(q, dtype=np.float64) - self.q0
        return 0.5 * (self.logdet_const + x @ self.prec @ x)

    def dVdq(self, q):
        return np.dot(self.prec, np.asarray(q, dtype=np.float64) - self.q0)


def probe_closures(D, V, dVdq, n_check=4, rtol=1e-9, seed=12345):
    """Recover an MVNTarget from the reference-style closures by affine probing."""
    z = np.zeros(D)
    g0 = np.asarray(dVdq(z), dtype=np.float64).reshape(-1)
    if g0.size != D:
        raise AssertionError("dVdq must return a length-D vector")
    cols = np.empty((D, D))
    for i in range(D):
        e = np.zeros(D)
        e[i] = 1.0
        cols[:, i] = np.asarray(dVdq(e), dtype=np.float64).reshape(-1) - g0
    P = cols
    if not np.any(g0):
        q0 = np.zeros(D)
    else:
        q0 = -np.linalg.solve(P, g0)
    logc = 2.0 * float(V(q0))
    t = MVNTarget(q0, prec=P, logdet_const=logc)
    rng = np.random.RandomState(seed)           # private stream: never touches the global np.random
    for _ in range(n_check):
        x = q0 + rng.standard_normal(D) * 1.7
        g_ref = np.asarray(dVdq(x), dtype=np.float64).reshape(-1)
        g = t.dVdq(x)
        if not np.allclose(g, g_ref, rtol=rtol, atol=rtol * (1 + np.abs(g_ref).max())):
            raise NotImplementedError("dVdq is not affine: the GPU engine supports multivariate-normal "
                                      "targets only (pass target=MVNTarget(q0, cov0))")
        v_ref = float(V(x))
        if not np.isclose(t.V(x), v_ref, rtol=rtol, atol=rtol * (1 + abs(v_ref))):
            raise NotImplementedError("V is not the MVN potential matching dVdq (pass target=MVNTarget)")
    return t
