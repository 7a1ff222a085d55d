"""HMC_sampler — the reference's sampler-class surface, running on MI355X.

Mirror of jaekor91/understanding-HMC `samplers.py` (class `sampler`, :4-291, and
`HMC_sampler`, :297-924): same constructor signature and defaults, same
`gen_sample` / `compute_convergence_stats` entry points, same result attributes
(NumPy arrays of the same shapes and dtypes).  The chains run in the fused HIP
kernels of libhmc.so (understanding-hmc_amd/csrc); this module only prepares
device buffers and random streams and calls the C ABI.  There is no CPU engine.

Randomness (new optional kwarg `rng`):
  * "replay" (default): the momentum / trajectory-length / uniform draws are taken
    from the global legacy `np.random` in exactly the reference's order
    (samplers.py:415, :431, :441, :461 — SURVEY Q7) and replayed on the GPU, so
    with the same `np.random.seed` the results equal the reference's
    (bit-identical q_chain for diagonal targets in fp_mode="exact").
  * "philox": in-kernel Philox4x32-10 keyed by (seed, global chain id, iteration):
    for production sizes (the host streams would not fit); statistically
    equivalent, independent of launch geometry and GPU count.
"""
import time
import warnings

import numpy as np
import torch

from . import _lib as H
from .diagnostics import StreamingDiagnostics
from .engine import NutsEngine, RandomEngine
from .target import MVNTarget, probe_closures  # noqa: F401
from . import utils as U


def _dev_tensor(a, device, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(device)


class sampler(object):
    """Parent class (samplers.py:4-64): storage of chains and convergence stats."""

    def __init__(self, D, target_lnL, Nchain=2, Niter=1000, thin_rate=1, warm_up_num=0):
        self.D = D
        self.target_lnL = target_lnL
        self.Nchain = Nchain
        self.Niter = Niter
        self.thin_rate = thin_rate
        self.warm_up_num = warm_up_num
        self.L_chain = 1 + ((self.Niter - self.warm_up_num) // self.thin_rate)   # samplers.py:31
        if self.L_chain < 0:
            raise ValueError("negative dimensions are not allowed")             # np.zeros at :33
        self.q_chain = np.zeros((self.Nchain, self.L_chain, self.D), dtype=float)
        self.lnL_chain = np.zeros((self.Nchain, self.L_chain, 1))
        self.R_q = None
        self.R_lnL = None
        self.n_eff_q = None
        self.accept_R_warm_up = None
        self.accept_R = None
        self.dt_total = 0
        self.N_total_steps = 0

    def compute_convergence_stats(self):
        """samplers.py:53-64: stats over q_chain[:, 1:, :] (the first point is dropped, Q16).
        Computed on the device by the diagnostics kernels when the chain lives there."""
        src = getattr(self, "q_chain_device", None)
        if src is None:
            src = self.q_chain
        self.R_q, self.n_eff_q = U.convergence_stats(src[:, 1:, :], warm_up_num=0, thin_rate=1)
        return

    def plot_samples(self, title_prefix, show=False, savefig=False, xmax=None, dx=None, plot_normal=True,
                     plot_cov=True, q0=None, cov0=None):
        """samplers.py:67-291: the 3x3 summary figure, drawn on the host from the GPU results
        (hmc_amd.plots).  Returns the figure's numbers (plots.sample_summary)."""
        from . import plots
        return plots.plot_samples(self, title_prefix, show=show, savefig=savefig, xmax=xmax, dx=dx,
                                  plot_normal=plot_normal, plot_cov=plot_cov, q0=q0, cov0=cov0)


class HMC_sampler(sampler):
    """HMC sampler for a multivariate-normal target on MI355X (samplers.py:297-924).

    Extra optional kwargs (all new; defaults keep the reference behaviour):
      target   : MVNTarget; if None, V/dVdq are affine-probed (target.probe_closures)
      rng      : "replay" | "philox"
      seed     : Philox key (rng="philox")
      fp_mode  : "exact" (reference rounding, no FMA) | "fast" (FMA-contracted integrator)
      device   : torch device (default: current CUDA device)
      store_chain : keep the full (Nchain, L_chain, D) chain (default True).  False = streaming
                    mode: q_chain is None, R_q / n_eff_q come from on-device streamed sums
      stream_tmax, stream_feed : streaming mode's largest variogram lag and the iterations
                    between diagnostics updates
      iters_per_launch : iterations fused in one kernel launch (default: all)
      chain_offset : global id of this object's first chain (multi-GPU sharding)
    """

    def __init__(self, D, V, dVdq, Nchain=2, Niter=1000, thin_rate=1, warm_up_num=0,
                 cov_p=None, sampler_type="Fixed", L=None, global_dt=True, dt=None,
                 L_low=None, L_high=None, log2L=None, d_max=10, target=None, rng="replay", seed=0,
                 fp_mode="exact", device=None, store_chain=True, iters_per_launch=None, chain_offset=0,
                 stream_tmax=64, stream_feed=60):
        sampler.__init__(self, D=D, target_lnL=None, Nchain=Nchain, Niter=Niter, thin_rate=thin_rate,
                         warm_up_num=warm_up_num)
        self.V = V
        self.dVdq = dVdq
        assert (sampler_type == "Fixed") or (sampler_type == "Random") or (sampler_type == "NUTS") or \
            (sampler_type == "Static")                                            # samplers.py:331
        assert (dt is not None)                                                   # :332
        self.dt = dt
        self.global_dt = global_dt
        self.sampler_type = sampler_type
        if self.sampler_type == "Fixed":
            assert (L is not None)
            self.L = L
        elif self.sampler_type == "Random":
            assert (L_low is not None) and (L_high is not None)
            self.L_low = L_low
            self.L_high = L_high
        elif self.sampler_type == "Static":
            assert (log2L is not None)
            self.log2L = log2L
        elif self.sampler_type == "NUTS":
            assert d_max is not None
            self.d_max = d_max
        if cov_p is None:                                                         # :352-356
            self.cov_p = np.diag(np.ones(self.D))
        else:
            self.cov_p = cov_p
        self.inv_cov_p = np.linalg.inv(self.cov_p)
        self.E_chain = np.zeros((self.Nchain, self.L_chain, 1), dtype=float)     # :359-360
        self.dE_chain = np.zeros((self.Nchain, self.L_chain, 1), dtype=float)

        assert rng in ("replay", "philox")
        assert fp_mode in ("exact", "fast")
        self.rng = rng
        self.seed = int(seed)
        self.fp_mode = fp_mode
        self.store_chain = store_chain
        self.stream_tmax, self.stream_feed = int(stream_tmax), int(stream_feed)
        if not store_chain:
            self.q_chain = None
        self.iters_per_launch = iters_per_launch
        self.chain_offset = int(chain_offset)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._target = target
        self.n_leapfrog = 0
        self.q_chain_device = None

    # ------------------------------------------------------------------ target / descriptors
    def target(self):
        if self._target is None:
            self._target = probe_closures(self.D, self.V, self.dVdq)
        return self._target

    def _descriptors(self):
        t = self.target()
        dev = self.device
        keep = []
        cov_p = np.asarray(self.cov_p, dtype=np.float64)
        full_mass = bool(np.any(cov_p - np.diag(np.diag(cov_p))))
        diag = t.diagonal and not full_mass
        kind = H.HMC_TARGET_DIAG if diag else H.HMC_TARGET_DENSE
        q0 = None if t.zero_mean else _dev_tensor(t.q0, dev)
        if diag:
            prec = None if t.identity else _dev_tensor(np.diag(t.prec), dev)
        else:
            prec = _dev_tensor(t.prec, dev)
        minv_full = None
        if full_mass:                     # samplers.py:356, :835-837 with a full inv_cov_p
            minv = pscale = None
            minv_full = _dev_tensor(self.inv_cov_p, dev)
        else:
            minv_d = np.diag(self.inv_cov_p).astype(np.float64)
            ident_mass = np.all(np.diag(cov_p) == 1.0) and np.all(minv_d == 1.0)
            minv = None if ident_mass else _dev_tensor(minv_d, dev)
            pscale = None if ident_mass else _dev_tensor(np.sqrt(np.diag(cov_p)), dev)
        dt = np.asarray(self.dt, dtype=np.float64)
        if dt.ndim == 0:
            dtv, dts = None, float(dt)
        else:
            assert dt.size == self.D
            dtv, dts = _dev_tensor(dt.reshape(-1), dev), 0.0
        kick = None if minv_full is None else _dev_tensor(self.inv_cov_p @ np.asarray(t.prec, np.float64), dev)
        keep += [q0, prec, minv, pscale, dtv, minv_full, kick]
        T = H.Target(self.D, kind, H.ptr(q0), H.ptr(prec), t.logdet_const)
        K = H.Kinetic(H.ptr(minv), H.ptr(pscale), H.ptr(dtv), dts, H.ptr(minv_full), None, H.ptr(kick))
        return T, K, keep

    # ------------------------------------------------------------------ public API
    def gen_sample(self, q_start, N_save_chain0=0, verbose=True):
        """samplers.py:363-383: dispatch Random / NUTS; other types silently do nothing."""
        if self.sampler_type == "Random":
            self.gen_sample_random(q_start, N_save_chain0, verbose)
        elif self.sampler_type == "NUTS":
            self.gen_sample_NUTS(q_start, N_save_chain0, verbose)
        return

    def _replay_streams_random(self):
        """Draw p0, p, L, u from the global legacy np.random in the reference order (Q7):
        per chain: p0 (:415), then per iteration: p (:431), L (:441), u (:461)."""
        N, I, D = self.Nchain, self.Niter, self.D
        if N * I * D > (1 << 28):
            raise MemoryError("replay streams too large for the host; use rng='philox'")
        p0 = np.empty((N, D))
        P = np.empty((N, I, D))
        Ls = np.empty((N, I), dtype=np.int32)
        U_ = np.empty((N, I))
        ident = np.array_equal(self.cov_p, np.eye(D))
        zeros = np.zeros(D)
        for m in range(N):
            p0[m] = np.random.standard_normal(D) if ident else \
                np.random.multivariate_normal(zeros, self.cov_p, size=1)[0]
            for i in range(I):
                P[m, i] = np.random.standard_normal(D) if ident else \
                    np.random.multivariate_normal(zeros, self.cov_p, size=1)[0]
                Ls[m, i] = np.random.randint(low=self.L_low, high=self.L_high, size=1)[0]
                U_[m, i] = np.random.random(1)[0]
        with np.errstate(divide="ignore"):
            lnu = np.log(U_)
        return p0, P, Ls, lnu

    def gen_sample_random(self, q_start, N_save_chain0, verbose):
        """samplers.py:387-491 on the GPU (fused kernel hmc_random_iters via RandomEngine)."""
        q_start = np.asarray(q_start, dtype=np.float64)
        assert q_start.shape[0] == self.Nchain                                    # :396
        torch.cuda.set_device(self.device)
        n_save = int(N_save_chain0) if N_save_chain0 > 0 else 0
        eng = RandomEngine(self.target(), self.Nchain, self.Niter, self.warm_up_num, self.thin_rate, self.L_low,
                           self.L_high, self.dt, cov_p=self.cov_p, rng=self.rng, seed=self.seed,
                           fp_mode=self.fp_mode, chain_offset=self.chain_offset, store_chain=self.store_chain,
                           n_save=n_save, device=self.device)
        if self.rng == "replay":
            eng.set_replay(*self._replay_streams_random())
        t0 = time.time()
        eng.init(q_start.reshape(self.Nchain, self.D))
        self._run(eng)
        torch.cuda.synchronize(self.device)
        elapsed = time.time() - t0
        self._finish(eng, elapsed, verbose)
        print("Compute acceptance rate")                                         # :483-489
        if self.warm_up_num > 0:
            self.accept_R_warm_up = self._acc_wu / float(self.Nchain * self.warm_up_num)
            print("During warm up: %.3f" % self.accept_R_warm_up)
        self.accept_R = self._acc / float(self.Nchain * (self.Niter - self.warm_up_num + 1))
        print("After warm up: %.3f" % self.accept_R)
        print("Completed.")
        return

    def _run(self, eng):
        """All Niter iterations.  With store_chain the whole q_chain stays on the device and one
        launch covers `iters_per_launch` iterations (default: the whole run).  Without it
        (streaming mode) the rows go to a circular device window that feeds
        StreamingDiagnostics after every `stream_feed` iterations, so memory is
        O(Nchain * (stream_tmax + window) * D) and compute_convergence_stats() reads the
        streamed sums instead of a q_chain."""
        self._stream_diag = None
        if self.store_chain:
            step = self.iters_per_launch or self.Niter
            for it0 in range(1, self.Niter + 1, step):
                eng.run(it0, min(it0 + step, self.Niter + 1))
            return
        n_samples = self.L_chain - 1
        if n_samples < 4:
            raise AssertionError("streaming statistics need L_chain - 1 >= 4 samples per chain")
        tmax = next(t for t in (8, 16, 32, 64) if t >= min(int(self.stream_tmax), 64))   # kernel lag rings
        diag = StreamingDiagnostics(self.Nchain, self.D, n_samples, tmax=tmax, device=self.device)
        step = self.iters_per_launch or 20
        feed = max(step, (int(self.stream_feed) // step) * step)
        eng.run_streaming(diag, 1, self.Niter + 1, step, feed=feed)
        self._stream_diag = diag

    def compute_convergence_stats(self):
        """samplers.py:53-64.  In streaming mode (store_chain=False) the split-chain sums were
        accumulated on the device during the run: R-hat is exact, the ESS sum stops at lag
        stream_tmax if the reference's criterion has not fired by then."""
        diag = getattr(self, "_stream_diag", None)
        if diag is not None:
            self.R_q, self.n_eff_q = diag.finish()
            self.stream_info = dict(diag.info)
            if diag.info["truncated_dims"]:
                warnings.warn("streaming ESS: %d of %d dimensions need variogram lags beyond stream_tmax=%d; "
                              "their n_eff is the sum truncated there, not the reference's value.  The exact "
                              "estimator streams up to %s samples per chain (2*(stream_tmax + stream_feed/thin) "
                              "+ 1); this run has %d: raise stream_feed or store q_chain"
                              % (diag.info["truncated_dims"], self.D, diag.tmax, diag.info.get("exact_max_samples"),
                                 diag.info.get("n_samples", 0)), UserWarning, stacklevel=2)
            return
        sampler.compute_convergence_stats(self)

    def _finish(self, eng, elapsed, verbose):
        """Copy results to the reference's NumPy attributes and derive the counters."""
        c = eng.read_counters()
        if c[H.CNT_OOB_REJECT] > 0:
            raise IndexError("index out of bounds for q_chain during warm-up (reference samplers.py:471)")
        self._acc, self._acc_wu = int(c[H.CNT_ACCEPT]), int(c[H.CNT_ACCEPT_WU])
        self.n_leapfrog = int(c[H.CNT_LEAPFROG])
        N, D = self.Nchain, self.D
        self.N_total_steps += N * (1 + 2 * self.Niter) + D * int(c[H.CNT_LEAPFROG_SQ])   # Q13
        if verbose:
            self.dt_total += elapsed
            print("Ran %d chains on %s: %.2f s" % (N, self.device, elapsed))
        self.engine = eng
        self.q_chain_device = eng.q_chain
        self.q_device = eng.q
        if eng.q_chain is not None:
            self.q_chain = eng.q_chain.cpu().numpy()
        else:
            self.q_chain = None                     # streaming mode: statistics only
        self.E_chain = eng.E_chain.cpu().numpy()[:, :, None]
        self.dE_chain = eng.dE_chain.cpu().numpy()[:, :, None]
        if eng.n_save:
            n_save = eng.n_save
            self.decision_chain = np.zeros((n_save + 1, 1), dtype=int)
            self.decision_chain[:n_save, 0] = eng.decision.cpu().numpy()
            T_ = eng.traj.cpu().numpy()
            tl = eng.traj_len.cpu().numpy()
            self.phi_q = [T_[i, :tl[i]].copy() for i in range(n_save) if tl[i] > 0]

    def set_nuts_replay(self, p0, P, tape):
        """Explicit NUTS draw streams (rng="replay"): p0 (Nchain, D), p (Nchain, Niter, D) and a
        per-chain tape (Nchain, T) of the directions (:608) and uniforms (:750, :773) in the
        order the reference consumes them.  NUTS interleaves these draws with the data-dependent
        tree, so they cannot be pre-drawn from the global np.random; without a tape,
        rng="replay" NUTS runs the Philox streams keyed by a seed drawn from np.random (so
        np.random.seed still makes the run reproducible)."""
        self._nuts_replay = (np.asarray(p0, np.float64), np.asarray(P, np.float64), np.asarray(tape, np.float64))

    def gen_sample_NUTS(self, q_start, N_save_chain0, verbose, on_dmax="raise"):
        """samplers.py:495-808 on the GPU (hmc_nuts_iters via NutsEngine).  The reference's
        `assert False` at d > d_max-1 (:596-598) becomes AssertionError after the run
        (on_dmax="raise") or keeps the current sample (on_dmax="break")."""
        q_start = np.asarray(q_start, dtype=np.float64)
        assert q_start.shape[0] == self.Nchain                                    # :510
        if N_save_chain0 > 0:
            self.phi_q = []                                                       # :511-514 (never filled)
        torch.cuda.set_device(self.device)
        tape = getattr(self, "_nuts_replay", None)
        rng, seed = self.rng, self.seed
        if rng == "replay" and tape is None:
            # the reference draws directions and uniforms from np.random in a data-dependent order
            # (:608, :748, :773) that chain-parallel trees cannot follow: say that this run differs
            warnings.warn("NUTS rng='replay' without set_nuts_replay(): running Philox streams seeded "
                          "from np.random (reproducible, statistically equivalent, not the reference's "
                          "draws)", UserWarning, stacklevel=2)
            rng, seed = "philox", int(np.random.randint(0, 2 ** 62, dtype=np.int64))
        eng = NutsEngine(self.target(), self.Nchain, self.Niter, self.warm_up_num, self.thin_rate, self.d_max,
                         self.dt, cov_p=self.cov_p, rng=rng, seed=seed, fp_mode=self.fp_mode,
                         chain_offset=self.chain_offset, store_chain=self.store_chain, on_dmax=on_dmax,
                         device=self.device,
                         iters_per_call=(self.iters_per_launch or self.Niter) if self.store_chain
                         else (self.iters_per_launch or 20))                  # (_run's launch sizes)
        if rng == "replay":
            eng.set_replay(*tape)
        t0 = time.time()
        eng.init(q_start.reshape(self.Nchain, self.D))
        self._run(eng)
        torch.cuda.synchronize(self.device)
        elapsed = time.time() - t0
        c = eng.read_counters()
        if c[H.CNT_HANDOFF_GIVEUP] > 0:
            raise RuntimeError("NUTS kernel: %d chain hand-offs timed out" % c[H.CNT_HANDOFF_GIVEUP])
        if c[H.CNT_OOB_REJECT] > 0:
            raise IndexError("NUTS replay tape exhausted")
        if c[H.CNT_DMAX] > 0 and on_dmax == "raise":
            raise AssertionError("Doubling number d exceeds d_max = %d" % self.d_max)   # :596-598
        N, D = self.Nchain, self.D
        self.n_leapfrog = int(c[H.CNT_LEAPFROG])
        self.n_unstable = int(c[H.CNT_UNSTABLE])
        self.n_dmax = int(c[H.CNT_DMAX])
        self.N_total_steps += N * (1 + self.Niter) + (D + 1) * self.n_leapfrog  # :553, :570, :614-619, :640-644
        if verbose:
            self.dt_total += elapsed
            print("Ran %d NUTS chains on %s: %.2f s" % (N, self.device, elapsed))
        self.engine = eng
        self.q_chain_device = eng.q_chain
        self.q_device = eng.q
        self.q_chain = eng.q_chain.cpu().numpy() if eng.q_chain is not None else None
        self.E_chain = eng.E_chain.cpu().numpy()[:, :, None]
        self.dE_chain = eng.dE_chain.cpu().numpy()[:, :, None]
        print("Compute acceptance rate: By default equal to 1.")                 # :800-805
        if self.warm_up_num > 0:
            self.accept_R_warm_up = 1.
            print("During warm up: %.3f" % self.accept_R_warm_up)
        self.accept_R = 1.
        print("After warm up: %.3f" % self.accept_R)
        print("Completed.")
        return

    # ------------------------------------------------------------------ primitives (batched on GPU)
    def leap_frog(self, p_old, q_old):
        """samplers.py:831-839 for one (p, q) row or a batch of rows, on the GPU."""
        p = np.atleast_2d(np.asarray(p_old, dtype=np.float64))
        q = np.atleast_2d(np.asarray(q_old, dtype=np.float64))
        T, K, keep = self._descriptors()
        dev = self.device
        pt, qt = _dev_tensor(p, dev), _dev_tensor(q, dev)
        po, qo = torch.empty_like(pt), torch.empty_like(qt)
        stream = torch.cuda.current_stream(dev).cuda_stream
        H.check(H.lib().hmc_leapfrog(T, K, p.shape[0], H.ptr(pt), H.ptr(qt), H.ptr(po), H.ptr(qo),
                                     H.HMC_MODE_EXACT if self.fp_mode == "exact" else H.HMC_MODE_FAST,
                                     stream), "hmc_leapfrog")
        pn, qn = po.cpu().numpy(), qo.cpu().numpy()
        if np.ndim(p_old) == 1:
            return pn[0], qn[0]
        return pn, qn

    def E(self, q, p):
        """samplers.py:819-823 (V of utils.py:218 + K of :817) for one row or a batch."""
        qq = np.atleast_2d(np.asarray(q, dtype=np.float64))
        pp = np.atleast_2d(np.asarray(p, dtype=np.float64))
        T, K, keep = self._descriptors()
        dev = self.device
        qt, pt = _dev_tensor(qq, dev), _dev_tensor(pp, dev)
        Et = torch.empty(qq.shape[0], dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        H.check(H.lib().hmc_energy(T, K, qq.shape[0], H.ptr(qt), H.ptr(pt), H.ptr(Et), stream), "hmc_energy")
        E = Et.cpu().numpy()
        return E[0] if np.ndim(q) == 1 else E

    def K(self, p):
        """samplers.py:811-817 (host; tiny)."""
        return np.dot(p, np.dot(self.inv_cov_p, p)) / 2.

    def p_sample(self):
        """samplers.py:825-829 (host draw from the global legacy RNG, as the reference)."""
        return np.random.multivariate_normal(np.zeros(self.D), self.cov_p, size=1)

    def make_movie(self, title_prefix, q0=None, cov0=None, plot_cov=True, qmin=-3, qmax=3, **kwargs):
        """samplers.py:843-880: PNG deck of chain 0's captured trajectories (hmc_amd.plots)."""
        from . import plots
        return plots.make_movie(self, title_prefix, q0=q0, cov0=cov0, plot_cov=plot_cov, qmin=qmin, qmax=qmax,
                                **kwargs)

    def make_slide(self, title_prefix, idx, phi_q, q_accepted, decision, q0=None, cov0=None, plot_cov=False,
                   qmin=-3, qmax=3):
        """samplers.py:883-924."""
        from . import plots
        return plots.make_slide(title_prefix, idx, phi_q, q_accepted, decision, q0, cov0, plot_cov, qmin, qmax)
