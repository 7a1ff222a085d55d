"""Benchmark: leapfrog steps/s (whole job) + ESS/s of the many-chain Random-trajectory HMC on the
BASELINE.json metric configuration: D=100 unit MVN at 1,048,576 chains in total, fp64.

    python bench.py [--gpus N --steps K --warmup W]
        N > 1 without WORLD_SIZE: this process starts N ranks under torch.distributed.run (before
        any GPU call) and exits with their status; rank 0 prints the line.
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

--chains is the TOTAL over all ranks (default 1,048,576, the metric's "1M chains"); rank r takes a
contiguous global chain range.  Philox draws AND start points are keyed by the global chain id, so
every chain's samples are the same at any N: the N-GPU line is the same job as the 1-GPU line
(strong scaling).  --chains-per-gpu instead fixes the work per GPU (weak scaling; config c4).

--config picks a BASELINE.json configuration (explicit flags still override):
    metric  D=100 unit MVN, 1,048,576 chains in total (the default; BASELINE.json's metric)
    c1      case1-script.py shape: D=2 unit MVN, 10 chains, 1000 warm-up + 1000 timed iterations
    c2      D=100 unit MVN, 65,536 chains
    c3      D=100 rho=0.95 dense precision (MFMA gradient), 262,144 chains
    c4      D=1000 unit MVN, 131,072 chains per GPU (1,048,576 on 8 GPUs), streaming R-hat/ESS
    c5      NUTS, D=100 rho=0.95, 65,536 chains

One step = ONE kernel launch of hmc_random_iters that advances every chain of this GPU by
--iters-per-step HMC iterations (momentum resample, L ~ U{5..19} leapfrogs, Metropolis test, sample
row stored).  The timed launches store every q_chain row, E and dE (the reference's output
contract, samplers.py:436-471) into a circular device window of the last R rows (R <= K*S, sized to
--chain-budget-gb; 1M chains x 100 dims is 0.8 GB per row).  After the timed region the window
holds the last R samples of every chain; R-hat / ESS (reference estimator, utils.py:77-179) run on
them, and ESS/s = n_eff(R samples) / (time the timed loop spent producing R iterations).
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "understanding-hmc_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector = FP64 matrix peak (spec)
METRIC_CHAINS = 1 << 20      # BASELINE.json metric: "D=100 MVN at 1M chains"
DEBUG_ENV = ("HMC_DEBUG_ABLATE", "HMC_DEBUG_L", "HMC_DEBUG_STAMPS", "HMC_LIB_PATH", "HMC_AMD_LIB")


PRESETS = {
    "metric": dict(chains=METRIC_CHAINS, dim=100),
    "c1": dict(chains=10, dim=2, iters_per_step=100, steps=10, warmup=10),
    "c2": dict(chains=65536, dim=100),
    "c3": dict(chains=262144, dim=100, rho=0.95),
    "c4": dict(chains_per_gpu=131072, dim=1000, stream_diag=True),
    "c5": dict(chains=65536, dim=100, rho=0.95, sampler="nuts", steps=5, warmup=1),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric", choices=sorted(PRESETS),
                    help="BASELINE.json configuration preset (explicit flags override its values)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chains", type=int, default=METRIC_CHAINS,
                    help="chains in TOTAL, split over the ranks (default 1,048,576 = the metric's 1M chains)")
    ap.add_argument("--chains-per-gpu", type=int, default=0,
                    help="weak scaling: this many chains per rank (total = this x N); overrides --chains")
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--iters-per-step", type=int, default=0,
                    help="HMC iterations fused into one launch (= one timed step); 0 = auto: 40 for the Random "
                         "sampler (HMC_sampler.gen_sample fuses a whole run into one launch), 32 for NUTS (the Philox momenta of up to 32 iterations are drawn ahead per launch)")
    ap.add_argument("--chain-budget-gb", type=float, default=100.0,
                    help="HBM for the circular q_chain window of the timed launches (per GPU)")
    ap.add_argument("--fp-mode", default="fast", choices=["fast", "exact"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dt", type=float, default=0.1)
    ap.add_argument("--rho", type=float, default=0.0, help="MVN correlation (0: unit/diagonal kernel; "
                    ">0: dense precision, MFMA kernel, BASELINE config 3 uses 0.95 with 262144 chains)")
    ap.add_argument("--sampler", default="random", choices=["random", "nuts"],
                    help="nuts: BASELINE config 5 (use with --rho 0.95 --chains 65536)")
    ap.add_argument("--d-max", type=int, default=10)
    ap.add_argument("--cov-p-rho", type=float, default=0.0,
                    help="nuts: a full (non-diagonal) cov_p with this correlation (samplers.py:352-356; a "
                         "shape-range line, 6D^2 + 12D flops per leapfrog: P x, the kick inv_cov_p.P x, K)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget per process")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ess", action="store_true", help="no q_chain rows at all (ablation; not a metric line)")
    ap.add_argument("--stream-diag", action="store_true",
                    help="R-hat/ESS from streaming statistics fed INSIDE the timed loop over every timed sample "
                         "(config 4: D=1000)")
    ap.add_argument("--tmax", type=int, default=16, help="streaming variogram lags")
    ap.add_argument("--stream-feed", type=int, default=0,
                    help="--stream-diag: steps between diagnostics updates; 0 = auto: every ~200 iterations")
    ap.add_argument("--no-order-tiles", action="store_true",
                    help="dense targets: MFMA tiles in chain order instead of L-ordered tiles")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group of N > 1 runs: nccl (= RCCL over xGMI, one GPU per rank) or gloo "
                         "(host-side collectives; lets a test run several ranks on one GPU)")
    ap.add_argument("--no-telemetry", action="store_true", help="do not sample board power / shader clock")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / sharding check without a GPU: every rank joins a gloo group and reports "
                         "its global chain range; rank 0 prints them as one JSON line")
    pre, _ = ap.parse_known_args(argv)
    ap.set_defaults(**PRESETS[pre.config])
    a = ap.parse_args(argv)
    return a


def resolve_chains(a, world):
    """Total chains of the job and whether the per-GPU work is fixed (weak scaling)."""
    if a.chains_per_gpu > 0:
        return a.chains_per_gpu * world, True
    return a.chains, False


# ------------------------------------------------------------------ launcher (--gpus N, no torchrun)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """Start n ranks (one per GPU) under torch.distributed.run as a CHILD process and return its
    exit status.  Called before anything touches the GPU in this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def shard(total, world, rank):
    """Contiguous global chain range of `rank`: (offset, count); the first total % world ranks
    take one chain more."""
    base, extra = divmod(int(total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def window_rows(total_rows, budget_rows):
    """Rows R of the circular q_chain window: the largest divisor of total_rows that fits the
    budget, so that the last R timed rows end up in slot order 0..R-1 (row r at slot r % R)."""
    if total_rows <= budget_rows:
        return total_rows
    for r in range(max(1, budget_rows), 0, -1):
        if total_rows % r == 0:
            return r
    return 1


# ------------------------------------------------------------------ CPU baseline (oracle port)
def _cpu_worker(args):
    seed, D, budget, rho, sampler, d_max = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import hmc_oracle as O
    np.random.seed(seed)
    cov = np.eye(D) if rho == 0 else O.mvn_cov(D, rho)
    tgt = O.MVNTarget(np.zeros(D), cov)
    core = O.HMCCore(tgt, 0.1)
    q_start = O.start_pts(np.zeros(D), 2 * np.eye(D), 1)
    rnd = max(2, min(20, 2000 // D))       # iterations per round: D=1000 spends ~1 s per iteration
    lf = 0
    t0 = time.time()
    # rounds of iterations of the reference-equivalent engine until the budget is spent
    while time.time() - t0 < budget:
        if sampler == "nuts":
            out = O.gen_sample_nuts(core, q_start, 1, 2, 0, 1, d_max, O.LiveDraws(D, np.eye(D)), on_dmax="break")
        else:
            out = O.gen_sample_random(core, q_start, 1, rnd, 0, 1, 5, 20, O.LiveDraws(D, np.eye(D)))
        lf += out["n_leapfrog"]
        q_start = out["q_chain"][:, -1, :]
    return lf, time.time() - t0


def host_cores():
    """(cores used, affinity cores, cgroup quota cores or None): processes = affinity cores,
    capped only by the cgroup CPU quota (running more processes than the quota grants would
    report a time-sliced, not a per-core, rate)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(D, budget, rho=0.0, sampler="random", d_max=10):
    procs, aff, quota = host_cores()
    env_threads = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in env_threads:
        os.environ[k] = "1"
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(1000 + i, D, budget, rho, sampler, d_max) for i in range(procs)])
    for k, v in env_threads.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    lf = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return dict(value=lf / wall, unit="leapfrog steps/s", cores=procs, kind="port",
                per_core=lf / wall / procs, cpu_model=cpu_model(), affinity_cores=aff, cgroup_quota_cores=quota,
                sample=f"oracle/hmc_oracle.py {sampler} engine (reference-equivalent NumPy: eigh logpdf per E, "
                       f"SVD mvn per draw), D={D} rho={rho}, {procs} procs x 1 chain x ~{budget:.0f} s, one BLAS "
                       f"thread each, {lf} leapfrogs")


# ------------------------------------------------------------------ profile-derived HBM traffic
def pmc_traffic(shape):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json),
    only when it was measured on this exact launch shape; None otherwise."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            entries = json.load(f)
    except (OSError, ValueError):
        return None
    for e in entries if isinstance(entries, list) else [entries]:
        if e.get("shape") == shape:
            return e
    return None


class Telemetry:
    """Board power and shader clock of this rank's GPU, sampled every `period` s by a host thread
    (amdsmi: read-only sysfs/SMU metrics, no HIP calls) while the timed region runs."""

    def __init__(self, index, period=0.01):
        self.index, self.period = index, period
        self.samples, self.error, self._th, self._stop = [], None, None, None

    def start(self):
        import threading
        try:
            import amdsmi as S
            S.amdsmi_init(S.AmdSmiInitFlags.INIT_AMD_GPUS)
            hs = S.amdsmi_get_processor_handles()
            self._h = hs[min(self.index, len(hs) - 1)]
            self._S = S
            self._read()
        except Exception as e:   # noqa: BLE001 (telemetry is optional: report why it is missing)
            self.error = f"{type(e).__name__}: {e}"
            return self
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._loop, daemon=True)
        self._th.start()
        return self

    def _read(self):
        S = self._S
        pw = S.amdsmi_get_power_info(self._h)
        ck = S.amdsmi_get_clock_info(self._h, S.AmdSmiClkType.GFX)
        w = pw.get("current_socket_power")
        if not isinstance(w, (int, float)):
            w = pw.get("average_socket_power")
        return (float(w) if isinstance(w, (int, float)) else None,
                float(ck["clk"]) if isinstance(ck.get("clk"), (int, float)) else None)

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._read())
            except Exception as e:   # noqa: BLE001
                self.error = f"{type(e).__name__}: {e}"
                return
            self._stop.wait(self.period)

    def stop(self):
        if self._th is not None:
            self._stop.set()
            self._th.join()
            try:
                self._S.amdsmi_shut_down()
            except Exception:   # noqa: BLE001
                pass
        w = [x[0] for x in self.samples if x[0] is not None]
        c = [x[1] for x in self.samples if x[1] is not None]
        return dict(power_W=float(np.mean(w)) if w else None, power_W_max=float(np.max(w)) if w else None,
                    sclk_MHz=float(np.mean(c)) if c else None, sclk_MHz_min=float(np.min(c)) if c else None,
                    samples=len(self.samples), source="amdsmi current_socket_power / GFX clock during the timed steps",
                    error=self.error)


def dry_run(a, world, rank):
    """The rank/offset logic of a real run, on CPU ranks (gloo): no GPU is touched."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    total, weak = resolve_chains(a, world)
    offset, count = shard(total, world, rank)
    mine = torch.tensor([rank, offset, count], dtype=torch.int64)
    got = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(got, mine)
    else:
        got = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "config": a.config, "n_gpus": world, "chains_total": total,
                          "scaling": "weak" if weak else "strong", "dim": a.dim,
                          "shards": [[int(v) for v in g] for g in got]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    for k in DEBUG_ENV:
        if os.environ.get(k):
            raise SystemExit(f"bench.py: {k} is set; debug/override variables are not allowed in a bench run")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    world = int(world_env or "1")
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    if a.dry_run:
        return dry_run(a, world, rank)
    # one GPU per rank; with fewer GPUs than ranks (a gloo test on a 1-GPU box) ranks share them
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from hmc_amd.engine import NutsEngine, RandomEngine
    from hmc_amd.target import MVNTarget
    from hmc_amd import _lib as H
    from hmc_amd.diagnostics import StreamingDiagnostics, convergence_stats
    from hmc_amd.utils import start_pts_device

    def reduce(vals, op):
        """Sum / max over ranks of a few host scalars."""
        t = torch.tensor(vals, dtype=torch.float64)
        if world > 1:
            t = t.to(dev) if a.backend == "nccl" else t
            dist.all_reduce(t, op=op)
        return t.cpu().numpy().tolist()

    nuts = a.sampler == "nuts"
    D = a.dim
    chains_total, weak = resolve_chains(a, world)
    offset, N = shard(chains_total, world, rank)
    S = a.iters_per_step if a.iters_per_step > 0 else (32 if nuts else (20 if a.stream_diag else 40))
    W, K = a.warmup, a.steps
    # streaming diagnostics fed every ~200 iterations: each feed re-reads the last tmax rows (the
    # variogram carry), so longer feeds cut the bytes per sample from (60+16+12)/60 to (200+16+12)/200
    # row reads, for a window of tmax + 200 + S + 2 rows (250 GB at c4's 131,072 x D=1000 per GPU;
    # profiles/r04_c4_feed_sweep.txt: feeds of 120 / 180 / 200 iterations 2.24e9 / 2.30e9 / 2.33e9)
    feed_steps = a.stream_feed if a.stream_feed > 0 else max(1, 200 // S)
    n_iter = (W + K) * S
    wu = W * S + 1                     # chain rows 0 .. K*S-1 are exactly the timed iterations
    timed_rows = K * S
    store = not (a.no_ess or a.stream_diag)
    # window rows from the per-GPU budget of the 1-GPU job (strong scaling) so that every N keeps
    # the same samples for R-hat / ESS; weak scaling: from this GPU's chains
    ref_chains = N if weak else chains_total
    R = window_rows(timed_rows, int(a.chain_budget_gb * 1e9 // (8.0 * max(1, ref_chains) * D))) if store else 0
    cov = np.eye(D) if a.rho == 0 else (np.diag(np.ones(D)) * (1 - a.rho) + a.rho)
    tgt = MVNTarget(np.zeros(D), cov)
    mass = nuts and a.cov_p_rho != 0
    if nuts:
        cov_p = (np.diag(np.ones(D)) * (1 - a.cov_p_rho) + a.cov_p_rho) if mass else None
        eng = NutsEngine(tgt, N, n_iter, wu, 1, a.d_max, a.dt, cov_p=cov_p, rng="philox", seed=a.seed,
                         fp_mode=a.fp_mode, chain_offset=offset, store_chain=False, on_dmax="break", device=dev,
                         iters_per_call=S)
    else:
        eng = RandomEngine(tgt, N, n_iter, wu, 1, 5, 20, a.dt, rng="philox", seed=a.seed, fp_mode=a.fp_mode,
                           chain_offset=offset, store_chain=False, device=dev, order_tiles=not a.no_order_tiles)
    window = None
    if store:                           # circular q_chain window: row r at slot r % R (every row stored)
        window = torch.zeros((N, R, D), dtype=torch.float64, device=dev)
        eng.set_chain_window(window, 0)
    sd = StreamingDiagnostics(N, D, eng.L_chain - 1, tmax=a.tmax, device=dev) if a.stream_diag else None
    # starts ~ N(0, 2I) keyed by the GLOBAL chain id (utils.py:204-209): the same job at any N
    eng.init(start_pts_device(a.seed, offset, N, D, scale=np.sqrt(2.0), device=dev))
    it = 1
    stream = torch.cuda.current_stream(dev)

    def step(i0, evs=None):
        if sd is not None:
            eng.run_streaming(sd, i0, i0 + S, S, events=evs, feed=S * feed_steps)
        else:
            if evs is not None:
                evs[0].record(stream)
            eng.run(i0, i0 + S)
            if evs is not None:
                evs[1].record(stream)

    for _ in range(W):
        step(it)
        it += S
    if window is not None and not a.no_ess and W > 0 and N >= 2:
        # warm-up of the post-run diagnostics too: the first launch of their kernels loads the code
        # object (~70 ms once per process); a 64-chain slice of the window has the same rows, so
        # the same lag-kernel instance (conv_tmax depends on the rows only).  Results discarded.
        convergence_stats(window[:min(N, 64)], warm_up_num=0, thin_rate=1)
    torch.cuda.synchronize(dev)
    c0 = eng.read_counters()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    tele = Telemetry(dev.index) if (rank == 0 and not a.no_telemetry) else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if tele is not None:
        tele.start()
    t0 = time.perf_counter()
    for k in range(K):
        step(it, ev[k])
        it += S
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    telemetry = tele.stop() if tele is not None else None
    elapsed = t1 - t0
    kern_ms = float(np.mean([s_.elapsed_time(e) for s_, e in ev]))
    c1 = eng.read_counters()
    lf_local = int(c1[H.CNT_LEAPFROG] - c0[H.CNT_LEAPFROG])
    acc = int(c1[H.CNT_ACCEPT] - c0[H.CNT_ACCEPT])
    if c1[H.CNT_HANDOFF_GIVEUP] > 0:
        raise RuntimeError("NUTS kernel: %d chain hand-offs timed out" % c1[H.CNT_HANDOFF_GIVEUP])
    dmax_hits = int(c1[H.CNT_DMAX] - c0[H.CNT_DMAX])
    wave_steps = int(c1[H.CNT_LEAPFROG_SQ] - c0[H.CNT_LEAPFROG_SQ])   # NUTS: steps of 16-chain waves
    lf_all, acc_all, dmax_all = reduce([float(lf_local), float(acc), float(dmax_hits)], dist.ReduceOp.SUM
                                       if world > 1 else None)
    t_max, kern_max = reduce([elapsed, kern_ms], dist.ReduceOp.MAX if world > 1 else None)
    value = lf_all / t_max
    ess = None
    if not a.no_ess:
        grp = dist.group.WORLD if world > 1 else None
        torch.cuda.synchronize(dev)
        td = time.perf_counter()
        if sd is not None:
            R_hat, neff = sd.finish(grp)
            n_samples, t_samples = K * S, t_max
        else:
            R_hat, neff = convergence_stats(window, warm_up_num=0, thin_rate=1, group=grp)
            n_samples, t_samples = R, t_max * R / float(timed_rows)
        torch.cuda.synchronize(dev)
        diag_s = time.perf_counter() - td
        from hmc_amd.diagnostics import LAST_INFO
        ess = dict(ess_per_s_median=float(np.median(neff)) / t_samples,
                   ess_per_s_min=float(np.min(neff)) / t_samples,
                   ess_per_s_median_incl_diag=float(np.median(neff)) / (t_samples + (0.0 if sd else diag_s)),
                   n_eff_median=float(np.median(neff)), n_eff_min=float(np.min(neff)),
                   rhat_median=float(np.median(R_hat)), rhat_max=float(np.max(R_hat)),
                   samples_per_chain=n_samples, sampling_s=t_samples, diagnostics_s=diag_s,
                   diagnostics_lags=dict(LAST_INFO),
                   method=(("reference estimator (every lag 1..n-1) over every timed sample: each split half "
                            "fed to the one-read lag kernel once complete, inside the timed loop"
                            if sd.mode == "exact" else
                            f"streaming statistics (tmax={a.tmax}) over every timed sample, fed inside the timed loop")
                           if sd is not None else
                           f"reference estimator on the circular window's last {R} samples per chain (all chains), "
                           f"after the timed loop; ESS/s = n_eff / time of the {R} iterations that produced them "
                           f"(ess_per_s_median_incl_diag adds the diagnostics' own time)"))
    if world > 1:
        dist.destroy_process_group()

    if rank == 0:
        dense = a.rho != 0 or nuts
        lf_launch = lf_local / K
        # kernel dispatches per timed step: the dense Random path with L-ordered tiles launches one
        # tile kernel per iteration (chains counting-sorted by that iteration's L); every other path
        # fuses the step's S iterations into one dispatch
        ordered = a.rho != 0 and not nuts and not a.no_order_tiles
        dispatches = S if ordered else 1
        # SURVEY.md §8(d) algorithmic bytes: 24*D + 24 per chain-iteration (read q, write q, write the
        # sample row, write E and dE) -- the unfused per-iteration contract
        bytes_model = N * S * (24 * D + 24)
        # what the step's dispatches must move: per chain-iteration one q_chain row + E + dE; q and
        # E_prev read and written once per dispatch
        row_bytes = 8 * D if (store or sd is not None) else 0
        bytes_moved = N * (S * (row_bytes + 16) + dispatches * (16 * D + 16))
        if dense:   # 2D^2 + 7D per leapfrog (Random dense), 2D^2 + 12D (NUTS: E + U-turn dots)
            # (a full cov_p: + 2D^2 for the kick inv_cov_p.(P x) and 2D^2 for K = p.inv_cov_p.p)
            flops_launch = lf_launch * ((6 if mass else 2) * D * D + (12 if nuts else 7) * D)
        else:       # 8D per leapfrog + 8D energies per iteration
            flops_launch = lf_launch * 8 * D + N * S * 8 * D
        kern_s = kern_ms / 1e3
        step_s = t_max / K
        tfl = flops_launch / kern_s / 1e12
        kname = "hmc_nuts_iters" if nuts else ("hmc_random_iters(dense)" if dense else "hmc_random_iters")
        shape = dict(kernel=kname, dim=D, chains_per_gpu=N, iters_per_step=S, window_rows=R,
                     stream_diag=bool(a.stream_diag), rho=a.rho)
        if mass:
            shape["cov_p_rho"] = a.cov_p_rho
        pm = pmc_traffic(shape)
        # PMC bytes are per hot-kernel DISPATCH (summarize_profile.py averages the timed dispatches);
        # kernel_ms times the step's dispatches together, so the step's traffic is dispatches x that
        traffic_dispatch = None if pm is None else pm["bytes_per_launch"]
        traffic = None if pm is None else traffic_dispatch * dispatches
        frac_meas = None if pm is None else traffic / kern_s / 1e9 / HBM_PEAK_GBS
        hbm = {"bound": "hbm", "achieved": bytes_model / kern_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": bytes_model / kern_s / 1e9 / HBM_PEAK_GBS,
               # what the fused dispatches must move (rows + E/dE + q and E_prev in and out per
               # dispatch) over the same time, next to the §8(d) model's unfused traffic above
               "frac_required": bytes_moved / kern_s / 1e9 / HBM_PEAK_GBS,
               "bytes_required_per_step": bytes_moved,
               "traffic": traffic, "traffic_per_dispatch": traffic_dispatch, "dispatches_per_step": dispatches,
               "traffic_source": None if pm is None else pm.get("source"),
               # measured HBM bytes (same-shape rocprofv3 PMC run) over the same kernel time
               "frac_measured": frac_meas,
               "kernel": kname, "kernel_ms": kern_ms, "bytes_per_launch": bytes_model, "shape": shape,
               "bytes_model": "SURVEY.md §8(d): (24*D + 24) B per chain-iteration x chains x iterations per step"}
        mfma = {"bound": "mfma" if dense else "fp64 vector", "achieved": tfl, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": tfl / FP64_PEAK_TFLOPS,
                "traffic": traffic, "traffic_per_dispatch": traffic_dispatch, "dispatches_per_step": dispatches,
                "traffic_source": None if pm is None else pm.get("source"),
                "shape": shape, "kernel": kname,
                "hbm_frac_measured": frac_meas,
                "kernel_ms": kern_ms, "flops_per_launch": flops_launch}
        if sd is not None:
            # the timed step also feeds the streaming diagnostics: `frac` above prices the sampler
            # launch alone (HIP events around it), frac_step the whole step `value` is timed on
            for r_ in (hbm, mfma):
                r_["step_ms"] = step_s * 1e3
            hbm["frac_step"] = bytes_model / step_s / 1e9 / HBM_PEAK_GBS
            mfma["frac_step"] = flops_launch / step_s / 1e12 / FP64_PEAK_TFLOPS
        roof = mfma if dense else hbm
        if telemetry is not None:
            roof["telemetry"] = telemetry
        tdesc = f"rho={a.rho} dense-precision MVN" if a.rho != 0 else "unit MVN"
        samp = f"NUTS d_max={a.d_max} (overflow counted, not aborted)" if nuts else "Random-L HMC, L~U{5..19}"
        if mass:
            samp += f", full cov_p (correlation {a.cov_p_rho})"
        store_desc = (f"every q_chain row, E, dE stored (circular window of {R} rows)" if store else
                      "rows fed to streaming diagnostics" if sd is not None else "no q_chain rows (ablation)")
        line = {
            "metric": "leapfrog steps/sec (whole node) + ESS/sec, D=100 MVN at 1M chains",
            "value": value,
            "unit": "leapfrog steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (D={D} {tdesc}, starts ~ N(0, 2I) keyed by global chain id, Philox4x32-10 draws)",
            "config": {"workload": f"{samp}, D={D} {tdesc}, dt={a.dt}, {chains_total} chains in total "
                                   f"({N} on rank 0), {S} iterations per step "
                                   + (f"({S} launches per step: one per iteration, L-ordered tiles)" if ordered
                                      else "(one fused launch)") +
                                   f", {store_desc}, fp_mode={a.fp_mode}",
                       "preset": a.config, "chains_total": chains_total, "chains_per_gpu": N, "dim": D,
                       "iters_per_step": S, "window_rows": R, "parallelism": f"chains{world}",
                       "backend": a.backend if world > 1 else None},
            "roofline": roof,
            "compute" if not dense else "memory": mfma if not dense else hbm,
            "leapfrogs": int(lf_all),
            "accepts": None if nuts else int(acc_all),
            "accept_rate": None if nuts else acc_all / (chains_total * K * S),
            "leapfrog_per_iteration": lf_all / (chains_total * K * S),
            "lane_utilisation": (lf_local / (16.0 * wave_steps)) if nuts and wave_steps else None,
            "dmax_fraction": (dmax_all / (chains_total * K * S)) if nuts else None,
            "debug_env_unset": True,
            "ess": ess,
        }
        if not a.no_cpu_baseline:       # rank 0 at any N, after every rank left the timed region
            line["cpu_baseline"] = cpu_baseline(D, a.cpu_seconds, a.rho, a.sampler, a.d_max)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
