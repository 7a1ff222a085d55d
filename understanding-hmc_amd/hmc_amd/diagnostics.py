"""Split-chain R-hat / ESS and per-dimension mean/std, computed on the GPU.

Same estimators as the reference (utils.py:77-179; samplers.py:213, :246),
including its quirks: W is the mean of per-split-chain *standard deviations*
(Q8) and the ESS early exit tests rho_1 twice (Q9).  Heavy sums run in the
libhmc.so diagnostics kernels; the O(D) combination and the ESS termination
loop (which only touches per-lag, per-dimension scalars) run on the host.

Multi-GPU: every sum is additive over chains, so with `group` (a
torch.distributed process group; RCCL over xGMI on MI355X) each rank reduces
its own chains and `all_reduce` combines the per-dimension sums.
"""
import numpy as np
import torch

from . import _lib as H

def _as_device(x):
    """(Nchain, T, D) float64 CUDA tensor view (no copy when already on the device)."""
    if isinstance(x, torch.Tensor):
        t = x if x.dtype == torch.float64 else x.double()
        if not t.is_cuda:
            t = t.cuda()
    else:
        t = torch.as_tensor(np.asarray(x, dtype=np.float64)).cuda()
    if t.stride(2) != 1:
        t = t.contiguous()
    return t


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _allreduce(x, group):
    """Sum over the ranks of `group` (RCCL over xGMI for device tensors; a gloo group -- CPU tests,
    or several ranks sharing one GPU -- reduces a host copy)."""
    if group is not None:
        if x.is_cuda and torch.distributed.get_backend(group) == "gloo":
            h = x.cpu()
            torch.distributed.all_reduce(h, group=group)
            x.copy_(h)
        else:
            torch.distributed.all_reduce(x, group=group)
    return x


class _Split:
    """Strided view of the split chains of convergence_stats (utils.py:88-104)."""

    def __init__(self, q_chain, thin_rate, warm_up_num):
        t = _as_device(q_chain)
        self.t = t
        Nchain, Niter, D = t.shape
        self.Nchain, self.D = Nchain, D
        Lt = len(range(warm_up_num, Niter, thin_rate))       # rows of q_chain[m, wu:][::thin]
        self.n = Lt // 2                                       # utils.py:102 (Py2 int division)
        self.ptr = t.data_ptr()                                # points at element [0, 0, 0] of the view
        self.base = warm_up_num * t.stride(1)
        self.cs = t.stride(0)
        self.ss = t.stride(1) * thin_rate


def split_moments(sp):
    L = H.lib()
    m2 = 2 * sp.Nchain
    mean = torch.empty((m2, sp.D), dtype=torch.float64, device=sp.t.device)
    std = torch.empty_like(mean)
    H.check(L.hmc_split_moments(sp.ptr, sp.Nchain, sp.cs, sp.ss, sp.base, sp.n, sp.D, H.ptr(mean), H.ptr(std),
                                _stream(sp.t)), "hmc_split_moments")
    return mean, std


def _rowsum(x2d, center=None):
    """Column sums of a contiguous (rows, D) device matrix (or of (x - center)^2)."""
    L = H.lib()
    rows, D = x2d.shape
    work = torch.empty(max(1, L.hmc_rowsum_work_size(rows, D)), dtype=torch.float64, device=x2d.device)
    out = torch.empty(D, dtype=torch.float64, device=x2d.device)
    H.check(L.hmc_rowsum(H.ptr(x2d), rows, D, 1, 0, 0, D, H.ptr(center), H.ptr(work), H.ptr(out),
                         _stream(x2d)), "hmc_rowsum")
    return out


def variogram_sums(sp, t0, t1):
    """sum_j sum_s (x_j[s+t]-x_j[s])^2 for t in [t0, t1) -> (t1-t0, D) device tensor."""
    L = H.lib()
    work = torch.empty(max(1, L.hmc_variogram_work_size(sp.Nchain, sp.D, t1 - t0)), dtype=torch.float64,
                       device=sp.t.device)
    out = torch.empty((t1 - t0, sp.D), dtype=torch.float64, device=sp.t.device)
    H.check(L.hmc_variogram(sp.ptr, sp.Nchain, sp.cs, sp.ss, sp.base, sp.n, sp.D, t0, t1, H.ptr(work), H.ptr(out),
                            _stream(sp.t)), "hmc_variogram")
    return out


def convergence_sums(sp, tmax):
    """One pass over the samples (C-ABI hmc_convergence_sums): (4 + tmax, D) device tensor of
    sum_j std_j, sum_j (mean_j - S), sum_j (mean_j - S)^2, the variogram sums of lags 1..tmax and
    that of lag n - 1, S = the view's first sample (see include/hmc.h)."""
    L = H.lib()
    work = torch.empty(max(1, L.hmc_convergence_work_size(sp.Nchain, sp.D, tmax)), dtype=torch.float64,
                       device=sp.t.device)
    out = torch.empty((4 + tmax, sp.D), dtype=torch.float64, device=sp.t.device)
    H.check(L.hmc_convergence_sums(sp.ptr, sp.Nchain, sp.cs, sp.ss, sp.base, sp.n, sp.D, tmax, H.ptr(work),
                                   H.ptr(out), _stream(sp.t)), "hmc_convergence_sums")
    return out


FIRST_PASS_LAGS = 96
COMPLETE_PASS_LAGS = 256


def conv_tmax(n):
    """Lags 1..tmax of the one-pass sums for split chains of n samples.  The pass always adds lag
    n - 1, so tmax = n - 2 makes it complete: every lag t < n, the whole ESS loop, in one read of the
    samples (the kernel's lag groups run to n - 1 - tail, the last tail <= 8 lags are summed in
    difference form).  Windows of up to COMPLETE_PASS_LAGS + 1 samples per half take that complete
    pass (n = 50, the bench window; n = 200, c3's: no second read whatever the mixing).  Longer
    chains take the first FIRST_PASS_LAGS lags; dimensions whose criterion has not fired by then
    read the remaining lags in ONE more pass (hmc_variogram), without the O(n^2) cost of every lag
    for fast-mixing ones."""
    if n - 1 <= COMPLETE_PASS_LAGS:
        return max(1, n - 2)
    return FIRST_PASS_LAGS


def _fits(cs, ss, n, D):
    """Whether the lag kernel's 32-bit buffer offsets cover a view (hmc_diag.hip lag_view_ok,
    pairs of halves): one chain's span must stay within 1 GiB."""
    if cs < n * ss:
        return False
    span = ((64 // D + 2) // 2 + 1) * cs + n * ss + D
    return (span + n * ss) * 8 < (1 << 30)


def _view_fits(sp):
    return _fits(sp.cs, sp.ss, sp.n, sp.D)


def rhat_ess_from_sums(sums, S, m_loc, n, tmax, group=None):
    """R-hat and the ESS loop (utils.py:109-157) from one-pass sums in the hmc_convergence_sums
    layout (sums (4 + tmax, D): sum_j std_j, sum_j (mean_j - S), sum_j (mean_j - S)^2, the variogram
    sums of lags 1..tmax, that of lag n - 1) over this rank's m_loc split chains, S their shift.
    Ranks all-reduce the per-dimension sums: two rounds, B needs the global mean.
    Returns (R numpy, n_eff numpy, need, Vt, var_h, m): `need` flags the dims whose criterion reads a
    lag beyond those given (n_eff NaN there), Vt the variogram values used."""
    D = sums.shape[1]
    dev = sums.device
    # round 1: sum_j std_j, sum_j mean_j (= shifted sum + m S), variogram sums, split-chain count
    r1 = torch.cat([sums[0:1], (sums[1] + m_loc * S)[None], sums[3:],
                    torch.full((1, D), float(m_loc), dtype=torch.float64, device=dev)])
    _allreduce(r1, group)
    m = int(round(float(r1[-1, 0].item())))
    assert m > 2                                                        # Nchain > 1, utils.py:85
    W = r1[0] / m                                                       # utils.py:112 (Q8)
    mean_all = r1[1] / m                                                # :119
    # round 2: sum_j (mean_j - mean_all)^2 from this rank's sums about its own shift S
    dS = S - mean_all
    bsum = _allreduce(sums[2] + 2.0 * dS * sums[1] + m_loc * dS * dS, group)
    B = bsum * n / float(m - 1)                                         # :120
    var = W * (n - 1) / float(n) + B / float(n)                         # :123
    R = torch.sqrt(var / W)                                             # :126
    v = r1[2:3 + tmax].cpu().numpy()                                    # lags 1..tmax, then lag n - 1
    var_h = var.cpu().numpy()
    # ---- ESS (utils.py:128-157), vectorised over dims
    lmax = max(n - 1, 2)                                                # lags t < n exist
    T = min(tmax, lmax)
    v = np.vstack([v[:T], v[tmax:tmax + 1]]) if T == n - 2 else v[:T]  # + lag n - 1: complete
    T = v.shape[0]
    Vt = v / (m * (n - np.arange(1, T + 1)))[:, None]                   # utils.py:177
    n_eff, need = ess_vectorised(Vt, var_h, n, m, complete=T >= lmax)
    return R.cpu().numpy(), n_eff, need, Vt, var_h, m


def convergence_stats(q_chain, thin_rate=5, warm_up_num=0, group=None):
    """utils.py:77-159 on the GPU.  q_chain: (Nchain, Niter, D) NumPy array or CUDA tensor
    (views such as q_chain_device[:, 1:, :] are read in place).  Returns (R, n_eff) NumPy.

    One pass over the samples gives every per-dimension sum R-hat needs and the variogram of every
    lag t < n up to conv_tmax(n), and of lag n - 1 (hmc_convergence_sums); the ESS termination
    (utils.py:130-157) runs vectorised over the dimensions on the host, and only dimensions whose
    criterion has not fired by then (long, slow-mixing windows) read the remaining lags, in one
    more pass (hmc_variogram).  Ranks all-reduce the per-dimension sums: two rounds, B needs the
    global mean.  Views whose chains span more than the lag kernel's 1 GiB offsets (very long stored
    runs) are processed as contiguous copies of dimension slices (every statistic is per dimension)."""
    sp = _Split(q_chain, thin_rate, warm_up_num)
    if not _view_fits(sp):
        return _convergence_stats_sliced(sp, thin_rate, warm_up_num, group)
    n, D = sp.n, sp.D
    dev = sp.t.device
    tmax = conv_tmax(n)
    sums = convergence_sums(sp, tmax)
    S = sp.t[0, warm_up_num, :].to(torch.float64)                       # the kernels' shift x[base + d]
    # (a strided view of the stored sample: no copy of a non-contiguous q_chain view, and the
    # right elements for dim-sliced views whose row stride is not D)
    R, n_eff, need, Vt, var_h, m = rhat_ess_from_sums(sums, S, 2 * sp.Nchain, n, tmax, group)
    lmax = max(n - 1, 2)
    LAST_INFO.clear()
    LAST_INFO.update(mode="stored", tmax=tmax, lags=Vt.shape[0], fallback_dims=int(need.sum()), fallback_passes=0,
                     truncated_dims=0)
    if need.any():
        # the dims whose criterion reads lags > T: gather their columns once (one strided read of
        # the lines holding them) into a compact (N, 2n, k) copy, and run the lag blocks on it (the
        # all-reduced sums make `need` the same on every rank)
        idx = np.nonzero(need)[0]
        if 4 * idx.size <= D:
            view = sp.t[:, warm_up_num::thin_rate, :][:, :2 * n, :]
            sub_t = view.index_select(2, torch.as_tensor(idx, device=dev)).contiguous()
            ssp = _Split(sub_t, 1, 0)
        else:                                    # most dims: read the samples in place instead
            ssp = sp
            idx = np.arange(D)
        Vs = Vt[:, idx]
        t0, t1 = Vs.shape[0] + 1, lmax + 1                              # every remaining lag t < n
        vb = _allreduce(variogram_sums(ssp, t0, t1), group).cpu().numpy()
        LAST_INFO["fallback_passes"] += 1
        lags = np.arange(t0, t1)
        Vs = np.vstack([Vs, vb / (m * (n - lags))[:, None]])
        ne, need2 = ess_vectorised(Vs, var_h[idx], n, m, complete=True)
        assert not need2.any()
        n_eff[idx] = ne
        LAST_INFO["lags"] = Vs.shape[0]
    return R, n_eff


def _convergence_stats_sliced(sp, thin_rate, warm_up_num, group):
    """convergence_stats of a view too long for the lag kernel's offsets: contiguous copies of
    dimension slices small enough to fit, each its own pass (R-hat and ESS are per dimension)."""
    t = sp.t
    N, L, D = t.shape
    rows = len(range(warm_up_num, L, thin_rate))
    per = D
    while per > 1 and not _fits(rows * per, per, rows // 2, per):     # a contiguous (N, rows, per) copy
        per = (per + 1) // 2
    if not _fits(rows * per, per, rows // 2, per):
        raise NotImplementedError("convergence_stats: %d samples per chain exceed the lag kernel's offsets" % rows)
    R, ne = np.empty(D), np.empty(D)
    info = None
    for d0 in range(0, D, per):
        d1 = min(D, d0 + per)
        sub = t[:, warm_up_num::thin_rate, d0:d1].contiguous()
        R[d0:d1], ne[d0:d1] = convergence_stats(sub, thin_rate=1, warm_up_num=0, group=group)
        info = dict(LAST_INFO) if info is None else {k: (info[k] + LAST_INFO[k] if k in ("fallback_dims",
                                                                                      "fallback_passes") else info[k])
                                                     for k in info}
    LAST_INFO.clear()
    LAST_INFO.update(info, slices=(D + per - 1) // per)
    return R, ne


LAST_INFO = {}   # what the last convergence_stats call read: fused lags, fallback dims and passes


def ess_vectorised(Vt, var, n, m, complete, truncate=False):
    """The termination loop of utils.py:130-157 for every dimension at once, given the variogram
    values Vt[t-1, d] = V_t of lags 1..T.  Returns (n_eff, need_more): a dimension whose criterion
    needs a lag beyond T while more lags exist (`complete` False) is flagged and its n_eff left
    NaN; truncate=True ends such sums at T instead (streaming windows).

    The reference loop (rho_k = 1 - V_k / (2 var)): if rho_1 < 0.01 (the Q9 test, sic) the sum is
    0; otherwise for t = 1 .. n-3 it appends rho_{t+2} and stops at the first ODD t with
    rho_{t+1} + rho_{t+2} < 0; the sum is rho_1 + ... + rho_t (t = n - 2 when it never stops,
    NaN propagating as in np.sum), clamped at 0; n_eff = m n / (1 + 2 sum)."""
    Vt = np.asarray(Vt, dtype=np.float64)
    T, D = Vt.shape
    with np.errstate(all="ignore"):
        rho = 1.0 - Vt / (2.0 * np.asarray(var, dtype=np.float64))[None, :]
        zero = rho[0] < 1e-2                                            # :136 (False for NaN)
        last = n - 3                                                    # the last t the loop checks
        avail = T - 2                                                   # checks whose lag t+2 we have
        ts = np.arange(1, min(last, avail) + 1, 2)
        t_stop = np.zeros(D, dtype=np.int64)
        if ts.size:
            hit = (rho[ts] + rho[ts + 1]) < 0                           # rho_{t+1} + rho_{t+2} < 0
            anyh = hit.any(axis=0)
            t_stop[anyh] = ts[hit.argmax(axis=0)[anyh]]
        if avail >= last or complete:
            t_none = max(n - 2, 1)                                      # ran to the end of the loop
        else:
            t_none = max(T - 1, 1) if truncate else 0                   # 0: more lags needed
        t = np.where(t_stop > 0, t_stop, t_none)
        need = ~zero & (t == 0)
        csum = np.cumsum(rho, axis=0)                                   # csum[t-1] = rho_1 + .. + rho_t
        ssum = csum[np.clip(t, 1, T) - 1, np.arange(D)]
        ssum = np.where(ssum < 0, 0.0, ssum)                            # :155-156 (NaN stays NaN)
        n_eff = np.where(zero, float(m * n), m * n / (1 + 2 * ssum))
    n_eff[need] = np.nan
    return n_eff, need


def _ess_dim(Vt, var, n, m, complete, truncate=False):
    """The termination loop of utils.py:130-157 given V_1..V_T (Vt[t-1]); None if more lags
    are needed (and not all lags are available yet).  truncate: the lags stop at len(Vt)
    (streaming window), the sum ends there."""
    def V(t):
        return Vt[t - 1] if t - 1 < len(Vt) else None
    v1, v2 = V(1), V(2)
    if v1 is None or (v2 is None and not complete):
        return None
    with np.errstate(all="ignore"):
        rho1 = 1. - v1 / (2 * var)
        rho2 = 1. - v2 / (2 * var) if v2 is not None else np.nan
    if (rho1 < 1e-2) or (rho1 < 1e-2):                                  # Q9 (sic)
        sum_rho = 0
    else:
        rho = [rho1, rho2]
        t = 1
        while t < n - 2:
            vt = V(t + 2)
            if vt is None:
                if truncate:
                    break
                return None
            rho.append(1 - vt / (2 * var))
            if ((t % 2) == 1) & ((rho[t] + rho[t + 1]) < 0):
                break
            t += 1
        sum_rho = np.sum(rho[:t])
        if sum_rho < 0:
            sum_rho = 0
    return m * n / (1 + 2 * sum_rho)


def variogram(chains, var_num, t_lag):
    """utils.py:161-179 for a list of (n, D) split chains (host arrays; API parity)."""
    m = len(chains)
    n = chains[0].shape[0]
    st = torch.as_tensor(np.stack([np.asarray(c, dtype=np.float64) for c in chains])).cuda()
    # treat each given chain as one "half": pair them as (2k, 2k+1) views of a (m/2, 2n, D) layout
    q = st.reshape(m, n, -1)
    sp = _Split.__new__(_Split)
    sp.t, sp.Nchain, sp.D, sp.n = q, (m + 1) // 2, q.shape[2], n
    sp.ptr, sp.base, sp.cs, sp.ss = q.data_ptr(), 0, 2 * n * q.shape[2], q.shape[2]
    if m % 2:
        raise AssertionError("variogram on an odd number of split chains is not supported on the GPU path")
    v = variogram_sums(sp, t_lag, t_lag + 1).cpu().numpy()[0, var_num]
    return v / float(m * (n - t_lag))


def per_dim_mean_std(q_chain, group=None):
    """np.mean / np.std over q_chain[:, 1:, i] per dimension (samplers.py:213, :246; Q16)."""
    t = _as_device(q_chain)
    N, T, D = t.shape
    L = H.lib()
    rows = N * (T - 1)
    work = torch.empty(max(1, L.hmc_rowsum_work_size(rows, D)), dtype=torch.float64, device=t.device)
    s = torch.empty(D, dtype=torch.float64, device=t.device)
    base = t.stride(1)
    H.check(L.hmc_rowsum(t.data_ptr(), N, t.stride(0), T - 1, t.stride(1), base, D, None, H.ptr(work), H.ptr(s),
                         _stream(t)), "hmc_rowsum")
    cnt = torch.tensor([float(rows)], dtype=torch.float64, device=t.device)
    _allreduce(s, group)
    _allreduce(cnt, group)
    mean = s / cnt
    m2 = torch.empty(D, dtype=torch.float64, device=t.device)
    H.check(L.hmc_rowsum(t.data_ptr(), N, t.stride(0), T - 1, t.stride(1), base, D, H.ptr(mean), H.ptr(work),
                         H.ptr(m2), _stream(t)), "hmc_rowsum")
    _allreduce(m2, group)
    std = torch.sqrt(m2 / cnt)
    return mean.cpu().numpy(), std.cpu().numpy()


# ---------------------------------------------------------------- streaming (windowed) statistics
def _colsum(x, center=None):
    """Per-dimension sum over the rows of a (rows, D) tensor (or of (x - center)^2): the HIP
    kernel for device tensors; torch on host tensors (the CPU multi-process path)."""
    if x.is_cuda:
        return _rowsum(x.contiguous(), center)
    return ((x - center) ** 2).sum(0) if center is not None else x.sum(0)


def combine_split_stats(mean, std, vsum, n, group=None, info=None):
    """R-hat and ESS (utils.py:109-157) from this rank's split-chain moments mean/std
    (m_local, D), its variogram lag sums vsum (T, D) (vsum[t-1] = sum over its split chains of
    sum_s (x[s+t] - x[s])^2, lags 1..T) and the half length n.  Every quantity is a sum over
    split chains, so ranks all-reduce them (two rounds: B needs the global mean).  Lags stop
    at T: the ESS sum ends there if the reference's criterion has not fired by then.  `info`
    (a dict) receives lags = T and truncated_dims = the number of dimensions whose reference
    loop (utils.py:139-152) would have read a lag beyond T: their n_eff is the sum truncated at
    T, not the reference's value."""
    dev = mean.device
    m = int(_allreduce(torch.tensor([float(mean.shape[0])], dtype=torch.float64, device=dev), group).item())
    assert m > 2                                                        # 2*Nchain, utils.py:85
    s1 = torch.stack([_colsum(std), _colsum(mean)])
    _allreduce(s1, group)
    W = s1[0] / m                                                       # utils.py:112 (Q8)
    mean_all = s1[1] / m                                                # :119
    bsum = _allreduce(_colsum(mean, center=mean_all), group)
    B = bsum * n / float(m - 1)                                         # :120
    var = W * (n - 1) / float(n) + B / float(n)                         # :123
    R = torch.sqrt(var / W)                                             # :126
    v = _allreduce(vsum.clone(), group).cpu().numpy()
    v = v[:max(2, min(v.shape[0], n - 1))]                              # lags t < n only
    T, D = v.shape
    lags = np.arange(1, T + 1)
    Vt = v / (m * (n - lags))[:, None]                                  # utils.py:177
    var_h = var.cpu().numpy()
    complete = T >= n - 1
    n_eff, _ = ess_vectorised(Vt, var_h, n, m, complete=complete, truncate=True)
    if info is not None:
        _, open_ = ess_vectorised(Vt, var_h, n, m, complete=complete, truncate=False)
        info.update(lags=int(T), truncated_dims=int(open_.sum()), n_half=int(n))
    return R.cpu().numpy(), n_eff


class StreamingDiagnostics:
    """convergence_stats (utils.py:77-159) of q_chain[:, 1:, :] without storing q_chain.

    Two modes, chosen by the sampler loop that feeds the rows (RandomEngine.run_streaming):
      * "exact": each split half is fed once it is complete and still whole in the circular window
        (add_half -> hmc_half_sums: the one-read lag kernel over that half of every chain, every lag
        1 .. n-1).  R-hat and ESS are then the reference estimator exactly (truncated_dims 0), and
        the window only has to hold one half plus a launch's rows.
      * "stream": halves longer than the window arrive in segments (update ->
        hmc_stream_accumulate): per-chain/half moments plus variogram lag sums for lags <= tmax.
        Exact for R-hat; the ESS sum stops at lag tmax where the reference's criterion has not
        fired by then (counted in info["truncated_dims"]).

    n_samples = L_chain - 1 (rows after the dropped first row, Q16)."""

    def __init__(self, n_chains, D, n_samples, tmax=16, device=None, mode=None):
        self.N, self.D, self.tmax = int(n_chains), int(D), int(tmax)
        self.n = int(n_samples) // 2                                    # utils.py:102
        assert self.n >= 2, "need at least 4 samples per chain"
        assert mode in (None, "exact", "stream")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self._z = lambda *s: torch.zeros(s, dtype=torch.float64, device=dev)  # noqa: E731
        self.pos = 0                                                    # samples consumed
        self.mode = mode                                                # "exact" | "stream"; None: the feeder picks
        self.window_rows = None                                         # rows of the feeder's window (first call)
        self.exact_max_samples = None                                   # feeder: largest n_samples fed exactly
        self._stream_state = None
        self.halves = []                                                # exact: halves added, in order
        self.xsums = None                                               # exact: sums about xshift
        self.xshift = None

    # stream-mode state, allocated on first use
    @property
    def shift(self):
        return self._state()[0]

    @property
    def s1(self):
        return self._state()[1]

    @property
    def s2(self):
        return self._state()[2]

    @property
    def vsum(self):
        return self._state()[3]

    def _state(self):
        if self._stream_state is None:
            N, D, z = self.N, self.D, self._z
            self.work = z(max(1, H.lib().hmc_stream_work_size(N, D, self.tmax)))
            self._stream_state = (z(N, 2, D), z(N, 2, D), z(N, 2, D), z(self.tmax, D))
        return self._stream_state

    def _set_mode(self, mode):
        if self.mode is None:
            self.mode = mode
        elif self.mode != mode:
            raise AssertionError("StreamingDiagnostics: a run feeds either whole halves or segments")

    def exact_lags(self):
        """tmax of the exact halves' sums: every lag 1 .. n-1 (n - 2 plus the lag n - 1 row)."""
        return max(1, self.n - 2)

    def add_half(self, window, h, slot0):
        """Exact mode: split half h (positions h*n .. h*n + n - 1) of every chain is complete in the
        circular window (N, W, D), its first sample in row slot0 (rows wrap at W).  One read of those
        rows gives its moments and every lag (hmc_half_sums), accumulated about a common shift."""
        self._set_mode("exact")
        assert window.stride(2) == 1 and window.shape[0] == self.N and window.shape[2] == self.D
        assert h == len(self.halves), "halves must be added in order"
        assert self.n <= window.shape[1], "the window must hold a whole half"
        T = self.exact_lags()
        L = H.lib()
        # (the kernels write every work entry they read: no zero fill)
        work = torch.empty(max(1, L.hmc_convergence_work_size(self.N, self.D, T)), dtype=torch.float64,
                           device=self.device)
        out = self._z(4 + T, self.D)
        Wr = window.shape[1]
        H.check(L.hmc_half_sums(window.data_ptr(), self.N, window.stride(0), window.stride(1), self.D, Wr,
                                int(slot0) % Wr, self.n, T, H.ptr(work), H.ptr(out), _stream(window)),
                "hmc_half_sums")
        S = window[0, int(slot0) % Wr, :].to(torch.float64).clone()     # the kernel's shift: chain 0's sample 0
        if self.xsums is None:
            self.xsums, self.xshift = out, S
        else:
            # re-centre onto the first half's shift: sum (mean - S0) = sum (mean - S) + N (S - S0), ...
            dS = S - self.xshift
            x = self.xsums
            x[2] += out[2] + 2.0 * dS * out[1] + self.N * dS * dS
            x[1] += out[1] + self.N * dS
            x[0] += out[0]
            x[3:] += out[3:]
        self.halves.append(h)
        self.pos = (h + 1) * self.n

    def update(self, window, carry, rows, slot0=0):
        """window: (N, W, D) device tensor (any chain/sample strides, dims contiguous), circular:
        the `carry` samples before the new ones and then the `rows` new samples sit in rows
        slot0, slot0 + 1, ... (mod W)."""
        assert window.stride(2) == 1 and window.shape[0] == self.N and window.shape[2] == self.D
        self._set_mode("stream")
        self._state()
        H.check(H.lib().hmc_stream_accumulate(window.data_ptr(), self.N, window.stride(0), window.stride(1), self.D,
                                              window.shape[1], int(slot0), int(carry), int(rows), self.pos, self.n,
                                              H.ptr(self.shift),
                                              H.ptr(self.s1), H.ptr(self.s2), self.tmax, H.ptr(self.work),
                                              H.ptr(self.vsum), _stream(window)), "hmc_stream_accumulate")
        self.pos += int(rows)

    def moments(self):
        """Split-chain means and stds (ddof=1), (2N, D), chain-major like split_moments."""
        n = float(self.n)
        mean = self.shift + self.s1 / n
        var = (self.s2 - self.s1 * self.s1 / n) / (n - 1.0)
        return mean.reshape(2 * self.N, self.D), torch.sqrt(torch.clamp(var, min=0.0)).reshape(2 * self.N, self.D)

    def finish(self, group=None):
        """(R, n_eff).  self.info (and diagnostics.LAST_INFO) then hold the mode, the lags used and
        truncated_dims: how many dimensions' ESS criterion had not fired by the last lag available,
        i.e. whose n_eff differs from the reference's (0 = every n_eff is the reference's; always 0
        in exact mode)."""
        assert self.pos >= 2 * self.n, "not all split-chain samples were fed"
        if self.mode == "exact":
            assert self.halves == [0, 1]
            T = self.exact_lags()
            R, n_eff, need, Vt, _, _ = rhat_ess_from_sums(self.xsums, self.xshift, 2 * self.N, self.n, T, group)
            assert not need.any()
            info = dict(mode="streaming-exact", lags=int(Vt.shape[0]), truncated_dims=0, n_half=int(self.n),
                        n_samples=2 * int(self.n), exact_max_samples=self.exact_max_samples)
            self.info = info
            LAST_INFO.clear()
            LAST_INFO.update(info)
            return R, n_eff
        mean, std = self.moments()
        info = dict(mode="streaming", tmax=self.tmax, n_half=int(self.n), n_samples=2 * int(self.n),
                    exact_max_samples=self.exact_max_samples)
        out = combine_split_stats(mean, std, self.vsum, self.n, group, info=info)
        self.info = info
        LAST_INFO.clear()
        LAST_INFO.update(info)
        return out
