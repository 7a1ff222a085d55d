"""Device-resident chain batch: buffers + C-ABI calls for the Random-trajectory sampler.

`RandomEngine` owns the (Nchain x D) state and the output arrays as torch CUDA
tensors (memory/streams only — all arithmetic is in libhmc.so) and exposes the
two calls of the hot path: `init()` (samplers.py:413-420) and `run(it0, it1)`
(iterations of samplers.py:428-475, fused in one kernel launch).  HMC_sampler
and bench.py are both thin layers over it.
"""
import hashlib
import json

import numpy as np
import torch

from . import _lib as H


def _dev(a, device, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(device)


class RandomEngine:
    def __init__(self, target, n_chains, n_iter, warm_up, thin, L_low, L_high, dt, cov_p=None, rng="philox",
                 seed=0, fp_mode="fast", chain_offset=0, store_chain=True, store_energy=True, n_save=0,
                 device=None, dense=False, order_tiles=True, random_ws=True):
        self.t = target
        self.D = D = target.D
        self.N = int(n_chains)
        self.n_iter, self.warm_up, self.thin = int(n_iter), int(warm_up), int(thin)
        self.L_chain = 1 + (self.n_iter - self.warm_up) // self.thin
        self.L_low, self.L_high = int(L_low), int(L_high)
        self.rng, self.seed, self.fp_mode = rng, int(seed), fp_mode
        self.chain_offset = int(chain_offset)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        dev = self.device
        # ---- target / kinetic descriptors (kept alive on the object)
        cov_p = np.diag(np.ones(D)) if cov_p is None else np.asarray(cov_p, dtype=np.float64)
        self.cov_p = cov_p
        full_mass = bool(np.any(cov_p - np.diag(np.diag(cov_p))))   # Q3 with a full cov_p
        diag = target.diagonal and not dense and not full_mass
        kind = H.HMC_TARGET_DIAG if diag else H.HMC_TARGET_DENSE
        self._q0 = None if target.zero_mean else _dev(target.q0, dev)
        if diag:
            self._prec = None if target.identity else _dev(np.diag(target.prec), dev)
        else:
            self._prec = _dev(target.prec, dev)
        self._minv_full = self._chol_t = self._kick = None
        if full_mass:
            # samplers.py:356 (inv_cov_p), :829 (p ~ N(0, cov_p) = C z) and :835-837 (kick by
            # inv_cov_p . dVdq): host-side constants of the run, like the reference's inv_cov_p
            minv_full = np.linalg.inv(cov_p)
            self._minv_full = _dev(minv_full, dev)
            self._chol_t = _dev(np.linalg.cholesky(cov_p).T, dev)
            self._kick = _dev(minv_full @ np.asarray(target.prec, dtype=np.float64), dev)
            self._minv = self._pscale = None
        else:
            minv = np.diag(np.linalg.inv(cov_p)).astype(np.float64)      # samplers.py:356
            ident_mass = bool(np.all(np.diag(cov_p) == 1.0) and np.all(minv == 1.0))
            self._minv = None if ident_mass else _dev(minv, dev)
            self._pscale = None if ident_mass else _dev(np.sqrt(np.diag(cov_p)), dev)
        dt = np.asarray(dt, dtype=np.float64)
        self.dt = dt
        if dt.ndim == 0:
            self._dtv, dts = None, float(dt)
        else:
            assert dt.size == D
            self._dtv, dts = _dev(dt.reshape(-1), dev), 0.0
        self.T = H.Target(D, kind, H.ptr(self._q0), H.ptr(self._prec), target.logdet_const)
        self.K = H.Kinetic(H.ptr(self._minv), H.ptr(self._pscale), H.ptr(self._dtv), dts, H.ptr(self._minv_full),
                           H.ptr(self._chol_t), H.ptr(self._kick))
        # ---- state and outputs
        N, Lc = self.N, self.L_chain
        self.q = torch.zeros((N, D), dtype=torch.float64, device=dev)
        self.E_prev = torch.zeros(N, dtype=torch.float64, device=dev)
        self.q_chain = torch.zeros((N, Lc, D), dtype=torch.float64, device=dev) if store_chain else None
        self.E_chain = torch.zeros((N, Lc), dtype=torch.float64, device=dev) if store_energy else None
        self.dE_chain = torch.zeros((N, Lc), dtype=torch.float64, device=dev) if store_energy else None
        self.counters = torch.zeros((H.COUNTER_SLOTS, H.NCOUNTERS), dtype=torch.int64, device=dev)
        self.n_save = int(n_save)
        if self.n_save:
            self.traj_stride = max(self.L_high, 1)
            self.traj = torch.zeros((self.n_save, self.traj_stride, 2), dtype=torch.float64, device=dev)
            self.traj_len = torch.zeros(self.n_save, dtype=torch.int32, device=dev)
            self.decision = torch.zeros(self.n_save, dtype=torch.int32, device=dev)
        else:
            self.traj_stride, self.traj, self.traj_len, self.decision = 0, None, None, None
        self.S = H.State(H.ptr(self.q), H.ptr(self.E_prev), H.ptr(self.q_chain), H.ptr(self.E_chain),
                         H.ptr(self.dE_chain), H.ptr(self.counters), H.ptr(self.traj), H.ptr(self.traj_len),
                         H.ptr(self.decision), self.n_save, self.traj_stride)
        # dense targets: scratch for L-ordered MFMA tiles (chains sorted by trajectory length
        # every iteration; same results, no lane idling through a longer trajectory).  The large-D
        # path (dense D > 128, diagonal D > 2048) keeps its chain state there: always allocated (a
        # NUTS run only needs it for hmc_chain_init's start energies, random_ws=False: sized for the
        # init alone, i.e. without the full-cov_p products unless cov_p is full)
        big = (D > 128) if kind == H.HMC_TARGET_DENSE else ((D + 1) // 2 > 16 * 64)
        L_ = H.lib()
        if big:
            nbytes = L_.hmc_random_workspace_size_ex(self.T, self.K, self.N)
        elif order_tiles and random_ws:
            nbytes = L_.hmc_random_workspace_size(self.T, self.N)
        else:
            nbytes = 0
        self._order = torch.zeros((nbytes + 3) // 4, dtype=torch.int32, device=dev) if nbytes > 0 else None
        self._order_bytes = self._order.numel() * 4 if self._order is not None else 0
        self.S.order = H.ptr(self._order)
        self._replay = None
        self._streams = []

    def set_chain_window(self, window, row0):
        """Store q_chain rows [row0, row0 + window.shape[1]) into `window` (N, W, D) instead of a
        whole-chain array (streaming diagnostics); other rows are not stored."""
        assert window.shape[0] == self.N and window.shape[2] == self.D and window.is_contiguous()
        self._window = window
        self.S.q_chain = window.data_ptr()
        self.S.qc_rows = window.shape[1]
        self.S.qc_row0 = int(row0)

    def set_replay(self, p0, P, Ls, lnu):
        """Host-replayed draws (rng='replay'): p0 (N,D), p (N,Niter,D), L (N,Niter), log u (N,Niter).
        L must lie in [L_low, L_high), the range np.random.randint draws it from (samplers.py:441):
        the kernels size trajectories (and the large-D path its launch count) by L_high."""
        Ls = np.asarray(Ls)
        if Ls.size and (Ls.min() < self.L_low or Ls.max() >= self.L_high):
            raise AssertionError("replay tape L outside [L_low, L_high) = [%d, %d)" % (self.L_low, self.L_high))
        dev = self.device
        self._streams = [_dev(p0, dev), _dev(P, dev), _dev(Ls, dev, torch.int32), _dev(lnu, dev)]
        self._replay = H.Replay(*[H.ptr(x) for x in self._streams], None, 0)

    d_max, on_dmax = 10, 0

    def schedule(self, it0, it1):
        return H.Schedule(self.N, self.chain_offset, self.n_iter, self.warm_up, self.thin, self.L_chain,
                          self.L_low, self.L_high, it0, it1,
                          H.HMC_RNG_REPLAY if self.rng == "replay" else H.HMC_RNG_PHILOX,
                          H.HMC_MODE_EXACT if self.fp_mode == "exact" else H.HMC_MODE_FAST, self.d_max,
                          self.on_dmax, self.seed)

    def stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def init(self, q_start):
        qs = q_start if isinstance(q_start, torch.Tensor) else _dev(np.asarray(q_start).reshape(self.N, self.D),
                                                                    self.device)
        self._qs = qs.to(self.device, torch.float64).contiguous()
        H.check(H.lib().hmc_chain_init_ws(self.T, self.K, self.schedule(1, 1), self._replay, H.ptr(self._qs), self.S,
                                          self._order_bytes, self.stream()), "hmc_chain_init")

    def run(self, it0, it1):
        """Iterations [it0, it1) of every chain in ONE fused kernel launch."""
        H.check(H.lib().hmc_random_iters_ws(self.T, self.K, self.schedule(it0, it1), self._replay, self.S,
                                            self._order_bytes, self.stream()), "hmc_random_iters")

    def run_streaming(self, diag, it_begin, it_end, step, events=None, feed=None):
        """Iterations [it_begin, it_end) in launches of `step`, with q_chain rows kept only in a
        circular device window (chain row r in window row r % W) that feeds `diag`
        (diagnostics.StreamingDiagnostics): memory O(N * (tmax + step/thin) * D) instead of
        O(N * L_chain * D), no copies.  Row 0 is not a sample of the statistics (Q16); rows are
        fed once complete (a thinned row is final after its last iteration).  May be called
        repeatedly with consecutive ranges and the same `step`.
        events: optional (start, end) CUDA events recorded around each sampler launch.
        feed: iterations between diagnostics updates (default `step`; a multiple of `step`).  Each
        update re-reads the last tmax rows (variogram carry), so feeding fewer, larger windows
        cuts the diagnostics' HBM traffic per sample from (rows + tmax + 12)/rows toward 1 row,
        for a window of tmax + (feed + step)/thin rows.  The last iteration always flushes."""
        N, D, T = self.N, self.D, diag.tmax
        feed = step if feed is None else int(feed)
        assert feed >= step and feed % step == 0, "feed must be a multiple of step"
        # exact mode (every lag of the reference's ESS loop) whenever a whole split half fits in no
        # more window than the segment mode would use: each half is fed once complete, from a
        # window of n + ceil(step/thin) + 2 rows; otherwise segments of `feed` iterations
        exact = diag.mode == "exact" or (diag.mode is None and diag.n <= T + feed // self.thin)
        W_seg = T + (feed + step) // self.thin + 2
        if exact:
            # both halves whole in the window (rows 1 .. 2n at slots 1 .. 2n: no half wraps, so the
            # lag pass reads plain strided rows) when that costs no more than the segment mode;
            # otherwise one half + a launch's rows, the second half wrapping
            W2 = 2 * diag.n + -(-step // self.thin) + 2
            W = W2 if W2 <= W_seg else diag.n + -(-step // self.thin) + 2
        else:
            W = W_seg
        # the mode and the window size are decided by the first call and recorded in `diag` (and
        # so in a checkpoint): a later call, or a resumed run, with another step or feed would
        # otherwise pick another mode or window size, and rows already written (the open half, the
        # variogram carry) would be silently replaced by a zeroed window (advisor r05)
        if diag.mode is None:
            diag._set_mode("exact" if exact else "stream")
            # the envelope of the exact mode for this feed: halves of n <= tmax + feed/thin samples
            diag.exact_max_samples = 2 * (T + feed // self.thin) + 1
        if diag.window_rows is not None and diag.window_rows != W:
            raise AssertionError("run_streaming continued with step/feed giving a %d-row window; the "
                                 "statistics' window has %d rows (use the same step and feed)" % (W, diag.window_rows))
        diag.window_rows = W
        st = getattr(self, "_stream", None)
        if st is None or st[0] is not diag or st[1].shape[1] != W:
            st = [diag, torch.zeros((N, W, D), dtype=torch.float64, device=self.device)]
            self._stream = st
        win = st[1]
        self.set_chain_window(win, 1)
        next_row = 1 + diag.pos            # next chain row the statistics need
        for a in range(it_begin, it_end, step):
            b = min(a + step, it_end)
            if events is not None:
                events[0].record(torch.cuda.current_stream(self.device))
            self.run(a, b)
            if events is not None:
                events[1].record(torch.cuda.current_stream(self.device))
            done = self.L_chain if b - 1 == self.n_iter else max(0, (b - self.warm_up) // self.thin)
            if exact:
                # split half h = chain rows 1 + h n .. (h + 1) n, whole in the window once complete
                h = len(diag.halves)
                while h < 2 and done >= 1 + (h + 1) * diag.n:
                    diag.add_half(win, h, (1 + h * diag.n) % W)
                    h += 1
                continue
            if done > next_row and (done - next_row >= feed // self.thin or b - 1 == self.n_iter):
                carry = min(T, next_row - 1)
                diag.update(win, carry, done - next_row, slot0=(next_row - carry) % W)
                next_row = done
        self.S.q_chain = H.ptr(self.q_chain)
        self.S.qc_rows = 0
        self.S.qc_row0 = 0

    # ---------------------------------------------------------------- checkpoint / resume
    def _meta(self):
        """Everything that decides the chain's next values: a checkpoint restores only into an
        engine with the same schedule, step size, mass matrix and target."""
        t = self.t
        h = hashlib.sha256()
        for a in (t.q0, t.prec, np.float64(t.logdet_const)):
            h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        return dict(kind=type(self).__name__, N=self.N, D=self.D, n_iter=self.n_iter, warm_up=self.warm_up,
                    thin=self.thin, L_chain=self.L_chain, L_low=self.L_low, L_high=self.L_high, seed=self.seed,
                    rng=self.rng, fp_mode=self.fp_mode, chain_offset=self.chain_offset, d_max=self.d_max,
                    order_tiles=self._order is not None,
                    dt=np.asarray(self.dt, dtype=np.float64).ravel().tolist(),
                    cov_p_sha256=hashlib.sha256(np.ascontiguousarray(self.cov_p, np.float64).tobytes()).hexdigest(),
                    target_sha256=h.hexdigest())

    def save(self, path, it_next, include_chain=True, diag=None):
        """Checkpoint after iteration it_next - 1 (.npz, no pickles).  Philox draws are keyed by
        (seed, global chain, iteration), so a run resumed from it_next reproduces the
        uninterrupted run bit for bit."""
        torch.cuda.synchronize(self.device)
        arr = dict(q=self.q, E_prev=self.E_prev, counters=self.counters)
        if include_chain and self.q_chain is not None:
            arr["q_chain"] = self.q_chain
        if self.E_chain is not None:
            arr["E_chain"], arr["dE_chain"] = self.E_chain, self.dE_chain
        if getattr(self, "ws", None) is not None:
            arr["ws"] = self.ws
        if self._order is not None:
            arr["order_ws"] = self._order                   # dense: tile order + gradient cache of q
        if diag is not None:
            if diag.mode == "exact":
                if diag.xsums is not None:
                    arr.update(diag_xsums=diag.xsums, diag_xshift=diag.xshift)
            else:
                arr.update(diag_shift=diag.shift, diag_s1=diag.s1, diag_s2=diag.s2, diag_vsum=diag.vsum)
            st = getattr(self, "_stream", None)
            if st is not None and st[0] is diag:
                arr["window"] = st[1]                       # rows of an open half / the lag carry
        meta = dict(self._meta(), it_next=int(it_next), diag_pos=None if diag is None else diag.pos,
                    diag_mode=None if diag is None else diag.mode,
                    diag_window_rows=None if diag is None else diag.window_rows,
                    diag_exact_max_samples=None if diag is None else diag.exact_max_samples,
                    diag_halves=None if diag is None else list(diag.halves))
        np.savez(path, meta=np.array(json.dumps(meta)), **{k: v.cpu().numpy() for k, v in arr.items()})

    def restore(self, path, diag=None):
        """Load a checkpoint written by save() into this (identically configured) engine;
        returns the iteration to continue from."""
        with np.load(path, allow_pickle=False) as z:
            meta = json.loads(str(z["meta"]))
            mine = self._meta()
            bad = {k: (meta.get(k), v) for k, v in mine.items() if meta.get(k) != v}
            if bad:
                raise AssertionError(f"checkpoint does not match this engine: {bad}")
            for k, t in (("q", self.q), ("E_prev", self.E_prev), ("counters", self.counters),
                         ("q_chain", self.q_chain), ("E_chain", self.E_chain), ("dE_chain", self.dE_chain),
                         ("ws", getattr(self, "ws", None)), ("order_ws", self._order)):
                if t is not None and k in z.files:
                    t.copy_(torch.as_tensor(z[k]).to(self.device))
            if self._order is not None and "order_ws" not in z.files:
                self._order.zero_()                         # no cached gradient: recomputed from q
            if diag is not None:
                diag.mode = meta.get("diag_mode")
                diag.window_rows = meta.get("diag_window_rows")
                diag.exact_max_samples = meta.get("diag_exact_max_samples")
                diag.halves = list(meta.get("diag_halves") or [])
                if diag.mode == "exact":
                    if "diag_xsums" in z.files:
                        diag.xsums = torch.as_tensor(z["diag_xsums"]).to(self.device)
                        diag.xshift = torch.as_tensor(z["diag_xshift"]).to(self.device)
                elif "diag_shift" in z.files:
                    for k, t in (("diag_shift", diag.shift), ("diag_s1", diag.s1), ("diag_s2", diag.s2),
                                 ("diag_vsum", diag.vsum)):
                        t.copy_(torch.as_tensor(z[k]).to(self.device))
                diag.pos = int(meta["diag_pos"])
                if "window" in z.files:
                    self._stream = [diag, torch.as_tensor(z["window"]).to(self.device)]
        return int(meta["it_next"])

    def read_counters(self):
        return self.counters.cpu().numpy().astype(np.int64).sum(axis=0)


class NutsEngine(RandomEngine):
    """Chain batch of the No-U-Turn sampler (samplers.py:495-808) on the dense-precision
    MFMA kernel (hmc_nuts_iters).  Diagonal targets are passed as dense precisions.
    `run(it0, it1)` advances every chain through iterations [it0, it1) in one launch; the
    tree workspace (live points, both ends, d_max+1 save slots per chain) stays on the device."""

    def __init__(self, target, n_chains, n_iter, warm_up, thin, d_max, dt, cov_p=None, rng="philox", seed=0,
                 fp_mode="fast", chain_offset=0, store_chain=True, store_energy=True, on_dmax="raise",
                 device=None, iters_per_call=None):
        # order_tiles=False: the NUTS kernel uses neither the tile order nor the gradient cache
        super().__init__(target, n_chains, n_iter, warm_up, thin, 5, 20, dt, cov_p=cov_p, rng=rng, seed=seed,
                         fp_mode=fp_mode, chain_offset=chain_offset, store_chain=store_chain,
                         store_energy=store_energy, n_save=0, device=device, dense=True, order_tiles=False,
                         random_ws=False)
        assert on_dmax in ("raise", "break")
        self.d_max = int(d_max)
        self.on_dmax = 0 if on_dmax == "raise" else 1
        # the Philox momenta drawn ahead are sized for the longest run() call (at most 32 iterations
        # are drawn per launch); replay tapes and a full cov_p draw in the kernel and need none
        self.iters_per_call = int(iters_per_call or n_iter)
        philox_mom = int(rng == "philox" and self._minv_full is None)
        nbytes = H.lib().hmc_nuts_workspace_size_ex(self.D, self.N, self.d_max, max(1, self.iters_per_call),
                                                    philox_mom)
        if nbytes <= 0:
            raise NotImplementedError("NUTS kernel: d_max=%d not supported (1 <= d_max <= 30)" % self.d_max)
        self.ws = torch.zeros((nbytes + 7) // 8, dtype=torch.float64, device=self.device)

    def set_replay(self, p0, P, tape):
        """Host-replayed draws: p0 (N,D), p (N,Niter,D), tape (N,T) directions/uniforms in order."""
        dev = self.device
        tape = np.ascontiguousarray(tape, dtype=np.float64)
        self._streams = [_dev(p0, dev), _dev(P, dev), _dev(tape, dev)]
        self._replay = H.Replay(H.ptr(self._streams[0]), H.ptr(self._streams[1]), None, None,
                                H.ptr(self._streams[2]), tape.shape[1])

    def run(self, it0, it1):
        if it1 - it0 > self.iters_per_call:
            raise ValueError("NutsEngine.run: %d iterations in one call, the workspace is sized for %d "
                             "(iters_per_call)" % (it1 - it0, self.iters_per_call))
        # the sized entry checks the workspace against what this call needs (include/hmc.h)
        H.check(H.lib().hmc_nuts_iters_ws(self.T, self.K, self.schedule(it0, it1), self._replay, self.S,
                                          H.ptr(self.ws), self.ws.numel() * 8, self.stream()), "hmc_nuts_iters_ws")
