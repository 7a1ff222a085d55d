"""CPU oracle: a clean-room NumPy restatement of the reference's HMC hot path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and there only as the
checker / the timed CPU baseline — never as the product path.  The product
(`understanding-hmc_amd/hmc_amd`) runs exclusively through the HIP C-ABI library.

Pinned: every function here is checked against golden vectors produced by the
reference itself (tests/golden/make_golden.py -> tests/golden/*.npz|json,
see tests/test_oracle.py).  Python 3 restatement of the Python-2 reference at
/root/reference (jaekor91/understanding-HMC); every function cites the
reference file:line it follows.  It keeps the reference's per-call cost
structure on purpose (scipy eigh-based logpdf per energy, numpy SVD-based
multivariate_normal per momentum draw, dense matvecs in every half kick), so
timing it is a fair stand-in for timing the reference.

Randomness: every engine takes a *draw source*.  `LiveDraws` consumes the
legacy global `np.random` in exactly the reference's order (samplers.py:415,
:431, :441, :461 / :565, :608, :748, :773); `ReplayDraws` replays recorded
streams (the golden fixtures, or the streams the product's replay mode feeds
the GPU).
"""
import numpy as np
from scipy.stats import multivariate_normal


# --------------------------------------------------------------------------- target
class MVNTarget:
    """V(q) = -log N(q; q0, cov0) and dVdq(q) = inv_cov0 (q - q0).

    Restates the driver closures of case1-script.py:26-49 (same in case2..5 and
    case3-script-2.py:27-50) and utils.normal_lnL (utils.py:213-218).
    """

    def __init__(self, q0, cov0):
        self.q0 = np.asarray(q0, dtype=np.float64)
        self.cov0 = np.asarray(cov0, dtype=np.float64)
        self.inv_cov0 = np.linalg.inv(self.cov0)           # case1-script.py:36

    def V(self, q):                                          # case1-script.py:39-43
        return -multivariate_normal.logpdf(q, mean=self.q0, cov=self.cov0)   # utils.py:218

    def dVdq(self, q):                                       # case1-script.py:45-49
        return np.dot(self.inv_cov0, (q - self.q0))


def mvn_cov(D, rho):
    """Sigma = (1-rho) I + rho 11^T  (case1-script.py:31-33)."""
    cov0 = np.diag(np.ones(D)) * (1 - rho)
    cov0 += rho
    return cov0


def start_pts(q0, cov0, size):
    """utils.py:204-209."""
    return np.random.multivariate_normal(q0, cov0, size=size)


# --------------------------------------------------------------------------- draws
class LiveDraws:
    """Draws from the legacy global np.random in the reference's call order."""

    def __init__(self, D, cov_p):
        self.D = D
        self.cov_p = cov_p

    def p(self, m, i):                 # samplers.py:825-829 (i = 0 -> the initial draw :415)
        return np.random.multivariate_normal(np.zeros(self.D), self.cov_p, size=1)[0]

    def L(self, m, i, lo, hi):         # samplers.py:441 (high exclusive, Q1)
        return np.random.randint(low=lo, high=hi, size=1)[0]

    def lnu(self, m, i):               # samplers.py:461
        return np.log(np.random.random(1))[0]

    # NUTS draws (samplers.py:608, :748, :773)
    def direction(self, m):
        return np.random.randint(low=0, high=2, size=1)[0]

    def uniform(self, m):
        return np.random.random()


class ReplayDraws:
    """Replays recorded streams: p0 (N,D), p (N,Niter,D), L (N,Niter), lnu (N,Niter);
    for NUTS a per-chain tape (N, T) of directions/uniforms in consumption order."""

    def __init__(self, p0, p, L=None, lnu=None, tape=None):
        self.p0, self.P, self.Ls, self.LNU = p0, p, L, lnu
        self.tape = tape
        self.tpos = None if tape is None else np.zeros(tape.shape[0], dtype=np.int64)

    def p(self, m, i):
        return self.p0[m] if i == 0 else self.P[m, i - 1]

    def L(self, m, i, lo, hi):
        return int(self.Ls[m, i - 1])

    def lnu(self, m, i):
        return self.LNU[m, i - 1]

    def _next(self, m):
        v = self.tape[m, self.tpos[m]]
        self.tpos[m] += 1
        return v

    def direction(self, m):
        return int(self._next(m))

    def uniform(self, m):
        return float(self._next(m))


# --------------------------------------------------------------------------- primitives
class HMCCore:
    """K, E, leap_frog of samplers.py:811-839 for a given target / mass / dt."""

    def __init__(self, target, dt, cov_p=None):
        self.t = target
        D = target.q0.size
        self.cov_p = np.diag(np.ones(D)) if cov_p is None else np.asarray(cov_p, np.float64)  # :352-355
        self.inv_cov_p = np.linalg.inv(self.cov_p)                                              # :356
        self.dt = dt

    def K(self, p):                                 # samplers.py:811-817
        return np.dot(p, np.dot(self.inv_cov_p, p)) / 2.

    def E(self, q, p):                              # samplers.py:819-823
        return self.t.V(q) + self.K(p)

    def leap_frog(self, p_old, q_old):              # samplers.py:831-839 (Q2, Q3)
        p_half = p_old - self.dt * np.dot(self.inv_cov_p, self.t.dVdq(q_old)) / 2.
        q_new = q_old + self.dt * p_half
        p_new = p_half - self.dt * np.dot(self.inv_cov_p, self.t.dVdq(q_new)) / 2.
        return p_new, q_new


def chain_len(Niter, warm_up, thin):
    """samplers.py:31."""
    return 1 + ((Niter - warm_up) // thin)


# --------------------------------------------------------------------------- Random engine
def gen_sample_random(core, q_start, Nchain, Niter, warm_up, thin, L_low, L_high, draws,
                      n_save_chain0=0):
    """Random-trajectory-length HMC, samplers.py:387-491.

    Chain-sequential, consuming `draws` in the reference order (Q7).  Returns a
    dict with the reference's result attributes.  Reproduces Q4 (initial draw
    used for E_chain[:,0] only), Q5 (negative-index q_chain writes during
    warm-up, IndexError when out of range), Q6 (acceptance denominators), Q13
    (N_total_steps += L*D inside the L loop) and Q14 (E/dE bookkeeping).
    """
    D = q_start.shape[1]
    assert q_start.shape[0] == Nchain                                   # :396
    Lc = chain_len(Niter, warm_up, thin)
    q_chain = np.zeros((Nchain, Lc, D))
    E_chain = np.zeros((Nchain, Lc))
    dE_chain = np.zeros((Nchain, Lc))
    save = n_save_chain0 > 0
    decision = np.zeros(n_save_chain0 + 1, dtype=np.int64) if save else None
    phi_q = [] if save else None
    acc_wu = acc = 0
    n_total = 0
    n_lf = 0
    for m in range(Nchain):                                              # :410
        q_chain[m, 0] = q_start[m]                                       # :413
        q_tmp = q_start[m]
        p_tmp = draws.p(m, 0)                                            # :415 (Q4)
        E_init = core.E(q_tmp, p_tmp)
        n_total += 1
        E_chain[m, 0] = E_init
        dE_chain[m, 0] = 0
        E_prev = E_init
        for i in range(1, Niter + 1):                                    # :428
            q_initial = q_tmp
            p_tmp = draws.p(m, i)                                        # :431
            E_init = core.E(q_tmp, p_tmp)                                # :434
            n_total += 1
            if i >= warm_up:                                             # :436-438 (Q14)
                r = (i - warm_up) // thin
                E_chain[m, r] = E_init
                dE_chain[m, r] = E_init - E_prev
            L = draws.L(m, i, L_low, L_high)                             # :441 (Q1)
            keep = save and m == 0 and i < n_save_chain0 + 1
            if keep:
                phi = np.zeros((L + 1, 2))
                phi[0] = q_tmp[:2]
            for l in range(1, L + 1):                                    # :448
                p_tmp, q_tmp = core.leap_frog(p_tmp, q_tmp)
                n_total += L * D                                         # :450 (Q13)
                if keep:
                    phi[l] = q_tmp[:2]
            n_lf += L
            E_final = core.E(q_tmp, p_tmp)                               # :455
            n_total += 1
            dE = E_final - E_init                                        # :459
            E_prev = E_init                                              # :460
            lnu = draws.lnu(m, i)                                        # :461
            if (dE < 0) or (lnu < -dE):                                  # :462
                if keep:
                    decision[i - 1] = 1
                if i >= warm_up:
                    q_chain[m, (i - warm_up) // thin] = q_tmp            # :466
                    acc += 1
                else:
                    acc_wu += 1
            else:
                r = (i - warm_up) // thin                                # :471 (Q5: may be negative)
                if r < -Lc:
                    raise IndexError("q_chain row %d out of range (reference samplers.py:471)" % r)
                q_chain[m, r] = q_initial
                q_tmp = q_initial
            if keep:
                phi_q.append(phi)
    out = dict(q_chain=q_chain, E_chain=E_chain, dE_chain=dE_chain, N_total_steps=n_total,
               n_leapfrog=n_lf, accept_R=acc / float(Nchain * (Niter - warm_up + 1)),
               accept_R_warm_up=(acc_wu / float(Nchain * warm_up)) if warm_up > 0 else None,
               accept_count=acc, accept_count_warm_up=acc_wu)
    if save:
        out["decision_chain"] = decision
        out["phi_q"] = phi_q
    return out


# --------------------------------------------------------------------------- NUTS bookkeeping
def find_next(table):
    """utils.py:222-228: first empty (-1) slot."""
    for i, e in enumerate(table):
        if e == -1:
            return i


def retrieve_save_index(table, l):
    """utils.py:230-237: slot holding point number l."""
    for i, m in enumerate(table):
        if m == l:
            return i


def check_points(m):
    """utils.py:246-283.  For even m: the first point of every aligned power-of-two
    sub-tree (size >= 2) that ends at m, smallest-start first.  Closed form: strip
    the leading bits of m until what remains (r) is a power of two (or r <= 2),
    then the points are start = m-r+1 and start + r/2 + r/4 + ... (>1 terms)."""
    assert m % 2 == 0
    r = int(m)
    while (r & (r - 1)) != 0 and r > 2:                # :262-265
        r -= 1 << (r.bit_length() - 1)
    start = m - r + 1                                   # :274
    pts = [start]
    tmp = start
    half = r
    while half > 2:                                      # :278-281 (pow_tmp > 1)
        half >>= 1
        tmp += half
        pts.append(tmp)
    return np.asarray(pts)


def release_fast(m, l):
    """utils.py:367-385 (same rule as release, :286-304)."""
    r_m, r_l = int(m), int(l)
    while (r_m & (r_m - 1)) != 0 and r_m > 4:           # :376-380
        top = 1 << (r_m.bit_length() - 1)
        r_m -= top
        r_l -= top
    return (r_m >= 4) and (r_l > 1)                      # :382


# --------------------------------------------------------------------------- NUTS engine
def gen_sample_nuts(core, q_start, Nchain, Niter, warm_up, thin, d_max, draws, on_dmax="raise"):
    """NUTS engine, samplers.py:495-808, restated.

    Quirks kept: Q10 (doubling continues until BOTH ends U-turn; a sub-tree is
    rejected only when both of its end checks fire), Q11 (biased sub-tree accept
    ratio exp(-(Emax_new-Emax_old))*pi_old/pi_new), Q12 (running-max energy
    normalisation; d >= d_max aborts), the |E-E0| > 1000 instability guard
    (:647-651) and accept_R hard-coded to 1 (:800-805).
    `on_dmax="raise"` reproduces the reference's assert (:596-598).
    """
    D = q_start.shape[1]
    assert q_start.shape[0] == Nchain
    Lc = chain_len(Niter, warm_up, thin)
    q_chain = np.zeros((Nchain, Lc, D))
    E_chain = np.zeros((Nchain, Lc))
    dE_chain = np.zeros((Nchain, Lc))
    q_save = np.zeros((d_max + 1, D))
    p_save = np.zeros((d_max + 1, D))
    table = np.ones(d_max + 1, dtype=int) * -1
    n_total = 0
    n_lf = 0
    n_unstable = 0
    for m in range(Nchain):
        q_chain[m, 0] = q_start[m]                                       # :548
        q_tmp = q_start[m]
        p_tmp = draws.p(m, 0)
        E_init = core.E(q_tmp, p_tmp)
        n_total += 1
        E_chain[m, 0] = E_init
        dE_chain[m, 0] = 0
        E_prev = E_init
        for i in range(1, Niter + 1):                                    # :563
            p_tmp = draws.p(m, i)                                        # :565
            E_init = core.E(q_tmp, p_tmp)                                # :569
            n_total += 1
            if i >= warm_up:
                r = (i - warm_up) // thin
                E_chain[m, r] = E_init
                dE_chain[m, r] = E_init - E_prev
            live_q_old = q_tmp                                           # :577
            left_q, left_p = q_tmp, -p_tmp                               # :581-584
            right_q, right_p = q_tmp, p_tmp
            E_max_old = E_init
            pi_old = 1
            left_term = right_term = False
            d = 0
            while (not left_term) or (not right_term):                   # :595 (Q10)
                if d > d_max - 1:                                        # :596-598 (Q12)
                    if on_dmax == "raise":
                        raise AssertionError("Doubling number d exceeds d_max = %d" % d_max)
                    break
                table[:] = -1                                            # :601
                L_new = 2 ** d
                u_dir = draws.direction(m)                               # :608
                if u_dir == 0:
                    p_tmp, q_tmp = core.leap_frog(right_p, right_q)
                else:
                    p_tmp, q_tmp = core.leap_frog(left_p, left_q)
                n_total += D
                n_lf += 1
                live_q_new = q_tmp                                       # :617
                E_max_now = core.E(q_tmp, p_tmp)                         # :618
                pi_new = 1
                n_total += 1
                s = find_next(table)                                     # :623-626
                q_save[s] = q_tmp
                p_save[s] = p_tmp
                table[s] = 1
                reject = False
                if L_new > 1:
                    for k in range(1, L_new):                            # :637
                        p_tmp, q_tmp = core.leap_frog(p_tmp, q_tmp)
                        n_total += D
                        n_lf += 1
                        E_tmp = core.E(q_tmp, p_tmp)                     # :643
                        n_total += 1
                        if np.abs(E_tmp - E_init) > 1000:                # :647-651
                            reject = True
                            q_tmp = live_q_old
                            n_unstable += 1
                            break
                        if ((k + 1) % 2) == 1:                           # :654-658
                            s = find_next(table)
                            q_save[s] = q_tmp
                            p_save[s] = p_tmp
                            table[s] = k + 1
                        else:
                            for l in check_points(k + 1):                # :699-736
                                s = retrieve_save_index(table, l)
                                q_chk = q_save[s]
                                p_chk = p_save[s]
                                if u_dir == 0:
                                    lq, lp, rq, rp = q_chk, -p_chk, q_tmp, p_tmp
                                else:
                                    lq, lp, rq, rp = q_tmp, p_tmp, q_chk, -p_chk
                                Dq = rq - lq
                                rt = np.dot(Dq, rp) < 0
                                lt = np.dot(-Dq, lp) < 0
                                if lt and rt:
                                    reject = True
                                    q_tmp = live_q_old
                                    break
                                if (l > 1) and release_fast(k + 1, l):
                                    table[s] = -1
                        if reject:
                            break
                        E_max_prev = E_max_now                           # :743-751
                        E_max_now = max(E_max_prev, E_tmp)
                        num = np.exp(-(E_tmp - E_max_now))
                        pi_new = num + np.exp(E_max_now - E_max_prev) * pi_new
                        r_ = num / pi_new
                        if draws.uniform(m) < r_:
                            live_q_new = q_tmp
                if reject:                                               # :754-755
                    break
                if u_dir == 0:                                           # :758-761
                    right_q, right_p = q_tmp, p_tmp
                else:
                    left_q, left_p = q_tmp, p_tmp
                r_ = np.exp(-(E_max_now - E_max_old)) * pi_old / pi_new  # :766 (Q11)
                E_max_old_prev = E_max_old
                E_max_old = max(E_max_old_prev, E_max_now)
                pi_old = (np.exp(-(E_max_now - E_max_old)) * pi_new
                          + np.exp(-(E_max_old_prev - E_max_old)) * pi_old)   # :771
                A = min(1, r_)
                if draws.uniform(m) < A:                                 # :773-775
                    live_q_old = live_q_new
                q_tmp = live_q_old                                       # :776
                Dq = right_q - left_q                                    # :779-781
                right_term = np.dot(Dq, right_p) < 0
                left_term = np.dot(-Dq, left_p) < 0
                d += 1
            E_prev = E_init                                              # :787
            if i >= warm_up:                                             # :790-791
                q_chain[m, (i - warm_up) // thin] = q_tmp
    return dict(q_chain=q_chain, E_chain=E_chain, dE_chain=dE_chain, N_total_steps=n_total,
                n_leapfrog=n_lf, n_unstable=n_unstable, accept_R=1.,
                accept_R_warm_up=1. if warm_up > 0 else None)


# --------------------------------------------------------------------------- diagnostics
def variogram(chains, var_num, t_lag):
    """utils.py:161-179 (BDA eq. 11.7)."""
    m = len(chains)
    n = chains[0].shape[0]
    V_t = 0.
    for c in chains:
        x = c[:, var_num]
        V_t += np.sum(np.square(x[t_lag:] - x[:-t_lag]))
    return V_t / float(m * (n - t_lag))


def split_chains(q_chain, thin_rate=5, warm_up_num=0):
    """utils.py:88-104: warm-up discard, thinning, even trim, split in halves."""
    chains = []
    n = None
    for m in range(q_chain.shape[0]):
        x = q_chain[m, warm_up_num:, :][::thin_rate, :]
        Lc = x.shape[0]
        if Lc % 2 != 0:
            x = x[:Lc - 1]
        n = Lc // 2            # utils.py:102 uses the *untrimmed* length (Py2 int division)
        chains.append(x[:n])
        chains.append(x[n:])
    return chains, n


def convergence_stats(q_chain, thin_rate=5, warm_up_num=0):
    """utils.py:77-159: split-chain R-hat (Q8: W = mean of std) and ESS (Q9)."""
    Nchain, Niter, D = q_chain.shape
    assert Nchain > 1                                                    # :85
    chains, n = split_chains(q_chain, thin_rate, warm_up_num)
    m = len(chains)
    W = np.mean(np.stack([np.std(c, ddof=1, axis=0) for c in chains]), axis=0)     # :109-112
    mw = np.stack([np.mean(c, axis=0) for c in chains])                              # :116-119
    mean_all = np.mean(mw, axis=0)
    B = np.sum(np.square(mw - mean_all), axis=0) * n / float(m - 1)                  # :120
    var = W * (n - 1) / float(n) + B / float(n)                                      # :123
    R = np.sqrt(var / W)                                                              # :126
    n_eff = np.zeros(D)
    for i in range(D):                                                               # :130-157
        rho1 = 1. - variogram(chains, i, 1) / (2 * var[i])
        rho2 = 1. - variogram(chains, i, 2) / (2 * var[i])
        if (rho1 < 1e-2) or (rho1 < 1e-2):                                          # :136 (Q9 typo kept)
            sum_rho = 0
        else:
            rho = [rho1, rho2]
            t = 1
            while t < n - 2:
                rho.append(1 - variogram(chains, i, t + 2) / (2 * var[i]))
                if ((t % 2) == 1) & ((rho[t] + rho[t + 1]) < 0):
                    break
                t += 1
            sum_rho = np.sum(rho[:t])
            if sum_rho < 0:
                sum_rho = 0
        n_eff[i] = m * n / (1 + 2 * sum_rho)
    return R, n_eff


def ess_from_variogram(var, Vt, n, m):
    """The ESS termination logic of utils.py:130-157 given precomputed variogram
    values Vt[t-1] = V_t (t = 1..T) for one dimension.  Used to check the
    product's device-side variogram sums; returns (n_eff, T_needed)."""
    rho1 = 1. - Vt[0] / (2 * var)
    rho2 = 1. - Vt[1] / (2 * var)
    if rho1 < 1e-2:
        return m * n / 1.0, 2
    rho = [rho1, rho2]
    t = 1
    while t < n - 2:
        rho.append(1 - Vt[t + 1] / (2 * var))
        if ((t % 2) == 1) & ((rho[t] + rho[t + 1]) < 0):
            break
        t += 1
    s = np.sum(rho[:t])
    if s < 0:
        s = 0
    return m * n / (1 + 2 * s), t + 2


def per_dim_mean_std(q_chain):
    """samplers.py:213 and :246: np.mean / np.std over q_chain[:, 1:, i] (Q16)."""
    x = q_chain[:, 1:, :]
    D = x.shape[2]
    return (np.array([np.mean(x[:, :, i]) for i in range(D)]),
            np.array([np.std(x[:, :, i]) for i in range(D)]))
