"""Host (NumPy) restatement of the draws the production Philox kernels consume.

Test infrastructure: the parity tests regenerate every random number a Philox-mode kernel
uses from the same counters and replay them through the oracle (oracle/hmc_oracle.py), so
that no test leans on the GPU's own generator for its expected values.

  * Philox4x32-10 (Salmon et al., SC'11): counter (slot, iteration, chain lo, chain hi), key
    (seed lo, seed hi); hmc_device.hpp::philox4x32_10.
  * Momentum pair k of iteration it >= 1 (dims 2k, 2k+1 for the diagonal kernels): the
    table-driven Box-Muller of hmc_device.hpp::normal_pair_tab, restated below with NumPy
    (1024-entry (cos, sin) and (1/c, -log 1/c) tables, the same bucket indices and series);
    iteration 0 (the initial momentum, samplers.py:415) uses hmc_device.hpp::normal_pair,
    i.e. plain Box-Muller on the same 52-bit uniforms.
  * Trajectory length (samplers.py:441) and MH log-uniform (:461): block (0x80000000,
    iteration, chain): L = L_low + (x * (L_high - L_low)) >> 32, u = u53(z, w).
The kernels' elementary functions are ~1 ulp; NumPy's are correctly rounded to ~0.5 ulp, so the
momenta agree to a few 1e-15 (checked against the C-ABI debug entry hmc_rng_normals in
tests/test_gpu_philox_parity.py), far inside the 1e-9 q tolerance of the parity tests.
"""
import numpy as np

KDRAW = 0x80000000
M32 = np.uint64(0xFFFFFFFF)
TAB_N = 1024


def np_philox(ctr, key):
    """Vectorised Philox4x32-10: ctr (n, 4) words, key (k0, k1) -> 4 uint64 arrays."""
    c = [ctr[:, i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    for _ in range(10):
        p0 = c[0] * np.uint64(0xD2511F53)
        p1 = c[2] * np.uint64(0xCD9E8D57)
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & M32, p1 & M32, ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & M32, p0 & M32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return c


def words(slot, it, gc, seed):
    """Philox blocks for counters (slot, it, gc): broadcast over array arguments."""
    slot, it, gc = np.broadcast_arrays(np.asarray(slot, np.uint64), np.asarray(it, np.uint64),
                                       np.asarray(gc, np.uint64))
    shape = slot.shape
    ctr = np.stack([slot.ravel(), it.ravel(), gc.ravel() & M32, gc.ravel() >> np.uint64(32)], axis=1)
    w = np_philox(ctr, (seed & 0xFFFFFFFF, seed >> 32))
    return [x.reshape(shape) for x in w]


def _mant52(lo, hi):
    """The 52-bit integer one_to_two() puts in the mantissa: (hi:lo) >> 12."""
    return (hi << np.uint64(20)) | (lo >> np.uint64(12))


def bm_pair(w):
    """hmc_device.hpp::normal_pair restated: Box-Muller on 52-bit uniforms."""
    a = _mant52(w[0], w[1]).astype(np.float64)
    b = _mant52(w[2], w[3]).astype(np.float64)
    r = np.sqrt(-2.0 * np.log(1.0 - a * 2.0 ** -52))
    ang = 2 * np.pi * (b * 2.0 ** -52)
    return r * np.cos(ang), r * np.sin(ang)


def _tables():
    i = np.arange(TAB_N, dtype=np.float64)
    trig_c, trig_s = np.cos(2 * np.pi * i / TAB_N), np.sin(2 * np.pi * i / TAB_N)
    c = 0.5 + (i + 0.5) * (0.5 / TAB_N)
    c[-1] = 1.0                                    # last bucket: log1p(m - 1), accurate near 1
    ic = 1.0 / c
    nlog = -np.log(ic)
    return trig_c, trig_s, ic, nlog


_TAB = _tables()


def table_pair(w):
    """hmc_device.hpp::normal_pair_tab restated: u1 = 1 - a 2^-52 in (0, 1] (exact),
    log u1 = k log 2 + L_j + log1p(m/c_j - 1) with bucket j = the top 10 mantissa bits of m,
    angle 2 pi b 2^-52 = table angle i (top 10 bits of b) + a remainder in [0, 2 pi/1024)."""
    trig_c, trig_s, ic, nlog = _TAB
    a = _mant52(w[0], w[1])
    u1 = 1.0 - a.astype(np.float64) * 2.0 ** -52
    m, k = np.frexp(u1)                             # u1 = m 2^k, m in [0.5, 1)
    j = ((m.view(np.uint64) >> np.uint64(42)) & np.uint64(TAB_N - 1)).astype(np.int64)
    r = m * ic[j] - 1.0                             # |r| <= 2^-11
    l1p = r + r * r * (-0.5 + r * (1.0 / 3 + r * (-0.25 + r * 0.2)))
    lg = k * np.log(2.0) + (nlog[j] + l1p)
    rad = np.sqrt(-2.0 * lg)
    b = _mant52(w[2], w[3])
    i = (b >> np.uint64(42)).astype(np.int64)
    f = (b & np.uint64((1 << 42) - 1)).astype(np.float64) * 2.0 ** -52
    dl = 2 * np.pi * f
    cd, sd = np.cos(dl), np.sin(dl)
    return rad * (trig_c[i] * cd - trig_s[i] * sd), rad * (trig_s[i] * cd + trig_c[i] * sd)


def u53(z, w):
    return ((w << np.uint64(21)) | (z >> np.uint64(11))).astype(np.float64) * 2.0 ** -53


def host_L_lnu(seed, gcs, niter, lo, hi):
    """(N, Niter) trajectory lengths and log-uniforms of iterations 1..Niter."""
    it = np.arange(1, niter + 1)[None, :]
    w = words(KDRAW, it, gcs[:, None], seed)
    L = lo + ((w[0] * np.uint64(hi - lo)) >> np.uint64(32)).astype(np.int64)
    u = u53(w[2], w[3])
    with np.errstate(divide="ignore"):
        lnu = np.log(u)
    return L.astype(np.int32), lnu


def table_normals(seed, chain0, n, it, npairs):
    """out[n][2*npairs]: the table Box-Muller normals of pairs 0..npairs-1 of iteration `it` for
    chains chain0 .. chain0+n-1 (the layout of the C-ABI entry hmc_rng_normals)."""
    gcs = np.arange(chain0, chain0 + n, dtype=np.uint64)
    z0, z1 = table_pair(words(np.arange(npairs)[None, :], it, gcs[:, None], seed))
    return np.stack([z0, z1], axis=2).reshape(n, 2 * npairs)


def wave_momenta(seed, N, D, niter, chain0=0, normals=table_normals):
    """Diagonal kernels: pair k holds dims 2k, 2k+1 (slot k).  p0 (iteration 0) from normal_pair,
    iterations >= 1 from the table transform (`normals`: the host restatement by default)."""
    npairs = (D + 1) // 2
    gcs = np.arange(chain0, chain0 + N, dtype=np.uint64)
    z0, z1 = bm_pair(words(np.arange(npairs)[None, :], 0, gcs[:, None], seed))
    p0 = np.stack([z0, z1], axis=2).reshape(N, 2 * npairs)[:, :D]
    P = np.stack([normals(seed, chain0, N, it, npairs)[:, :D] for it in range(1, niter + 1)], axis=1)
    return p0, P
