"""Benchmark: leapfrog steps/s (whole job) + ESS/s of the many-chain Random-trajectory HMC on the
BASELINE.json metric configuration: D=100 unit MVN at 1,048,576 chains in total, fp64.

    python bench.py [--gpus N --steps K --warmup W]
        N > 1 without WORLD_SIZE: this process starts N ranks under torch.distributed.run (before
        any GPU call) and exits with their status; rank 0 prints the line.
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

--chains is the TOTAL over all ranks (default 1,048,576, the metric's "1M chains"); rank r takes a
contiguous global chain range (Philox is keyed by the global chain id, so every chain's samples
are the same at any N).  The total is fixed, so scaling over N is strong scaling.

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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chains", type=int, default=METRIC_CHAINS,
                    help="chains in TOTAL, split over the ranks (default 1,048,576 = the metric's 1M chains)")
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--iters-per-step", type=int, default=0,
                    help="HMC iterations fused into one launch (= one timed step); 0 = auto: 40 for the Random "
                         "sampler (HMC_sampler.gen_sample fuses a whole run into one launch), 16 for NUTS")
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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget per process")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ess", action="store_true", help="no q_chain rows at all (ablation; not a metric line)")
    ap.add_argument("--stream-diag", action="store_true",
                    help="R-hat/ESS from streaming statistics fed INSIDE the timed loop over every timed sample "
                         "(config 4: D=1000)")
    ap.add_argument("--tmax", type=int, default=16, help="streaming variogram lags")
    ap.add_argument("--stream-feed", type=int, default=0,
                    help="--stream-diag: steps between diagnostics updates; 0 = auto: every ~60 iterations")
    ap.add_argument("--no-order-tiles", action="store_true",
                    help="dense targets: MFMA tiles in chain order instead of L-ordered tiles")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / sharding check without a GPU: every rank joins a gloo group and reports "
                         "its global chain range; rank 0 prints them as one JSON line")
    return ap.parse_args(argv)


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
    lf = 0
    t0 = time.time()
    # rounds of iterations of the reference-equivalent engine until the budget is spent
    while time.time() - t0 < budget:
        if sampler == "nuts":
            out = O.gen_sample_nuts(core, q_start, 1, 2, 0, 1, d_max, O.LiveDraws(D, np.eye(D)), on_dmax="break")
        else:
            out = O.gen_sample_random(core, q_start, 1, 20, 0, 1, 5, 20, O.LiveDraws(D, np.eye(D)))
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


def dry_run(a, world, rank):
    """The rank/offset logic of a real run, on CPU ranks (gloo): no GPU is touched."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    offset, count = shard(a.chains, world, rank)
    mine = torch.tensor([rank, offset, count], dtype=torch.int64)
    got = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(got, mine)
    else:
        got = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "chains_total": a.chains,
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
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from hmc_amd.engine import NutsEngine, RandomEngine
    from hmc_amd.target import MVNTarget
    from hmc_amd import _lib as H
    from hmc_amd.diagnostics import StreamingDiagnostics, convergence_stats

    nuts = a.sampler == "nuts"
    D = a.dim
    offset, N = shard(a.chains, world, rank)
    S = a.iters_per_step if a.iters_per_step > 0 else (16 if nuts else (20 if a.stream_diag else 40))
    W, K = a.warmup, a.steps
    feed_steps = a.stream_feed if a.stream_feed > 0 else max(1, 60 // S)
    n_iter = (W + K) * S
    wu = W * S + 1                     # chain rows 0 .. K*S-1 are exactly the timed iterations
    timed_rows = K * S
    store = not (a.no_ess or a.stream_diag)
    R = window_rows(timed_rows, int(a.chain_budget_gb * 1e9 // (8.0 * max(1, N) * D))) if store else 0
    cov = np.eye(D) if a.rho == 0 else (np.diag(np.ones(D)) * (1 - a.rho) + a.rho)
    tgt = MVNTarget(np.zeros(D), cov)
    if nuts:
        eng = NutsEngine(tgt, N, n_iter, wu, 1, a.d_max, a.dt, rng="philox", seed=a.seed, fp_mode=a.fp_mode,
                         chain_offset=offset, store_chain=False, on_dmax="break", device=dev)
    else:
        eng = RandomEngine(tgt, N, n_iter, wu, 1, 5, 20, a.dt, rng="philox", seed=a.seed, fp_mode=a.fp_mode,
                           chain_offset=offset, store_chain=False, device=dev, order_tiles=not a.no_order_tiles)
    window = None
    if store:                           # circular q_chain window: row r at slot r % R (every row stored)
        window = torch.zeros((N, R, D), dtype=torch.float64, device=dev)
        eng.set_chain_window(window, 0)
    sd = StreamingDiagnostics(N, D, eng.L_chain - 1, tmax=a.tmax, device=dev) if a.stream_diag else None
    rs = np.random.RandomState(a.seed + rank)
    eng.init(torch.as_tensor(rs.standard_normal((N, D)) * np.sqrt(2.0), device=dev))
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
    torch.cuda.synchronize(dev)
    c0 = eng.read_counters()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        step(it, ev[k])
        it += S
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    c1 = eng.read_counters()
    lf_local = int(c1[H.CNT_LEAPFROG] - c0[H.CNT_LEAPFROG])
    acc = int(c1[H.CNT_ACCEPT] - c0[H.CNT_ACCEPT])
    if a.sampler == "nuts" and c1[H.CNT_ACCEPT] > 0:   # NUTS uses this slot for chain hand-off give-ups
        raise RuntimeError("NUTS kernel: %d chain hand-offs timed out" % c1[H.CNT_ACCEPT])
    dmax_hits = int(c1[H.CNT_DMAX] - c0[H.CNT_DMAX])
    wave_steps = int(c1[H.CNT_LEAPFROG_SQ] - c0[H.CNT_LEAPFROG_SQ])   # NUTS: steps of 16-chain waves
    tot = torch.tensor([float(lf_local), float(acc), float(dmax_hits), elapsed, kern_ms], dtype=torch.float64,
                       device=dev)
    if world > 1:
        s = tot[:3].clone()
        dist.all_reduce(s)
        m = tot[3:].clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot = torch.cat([s, m])
    lf_all, acc_all, dmax_all, t_max, kern_max = tot.cpu().numpy().tolist()
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
        ess = dict(ess_per_s_median=float(np.median(neff)) / t_samples,
                   ess_per_s_min=float(np.min(neff)) / t_samples,
                   n_eff_median=float(np.median(neff)), n_eff_min=float(np.min(neff)),
                   rhat_median=float(np.median(R_hat)), rhat_max=float(np.max(R_hat)),
                   samples_per_chain=n_samples, sampling_s=t_samples, diagnostics_s=diag_s,
                   method=(f"streaming statistics (tmax={a.tmax}) over every timed sample, fed inside the timed loop"
                           if sd is not None else
                           f"reference estimator on the circular window's last {R} samples per chain (all chains), "
                           f"after the timed loop; ESS/s = n_eff / time of the {R} iterations that produced them"))

    if rank == 0:
        dense = a.rho != 0 or nuts
        lf_launch = lf_local / K
        # SURVEY.md §8(d) algorithmic bytes: 24*D + 24 per chain-iteration (read q, write q, write the
        # sample row, write E and dE) -- the unfused per-iteration contract
        bytes_model = N * S * (24 * D + 24)
        # what the fused launch must move: per chain-iteration one q_chain row + E + dE; q and E_prev
        # read and written once per launch
        row_bytes = 8 * D if (store or sd is not None) else 0
        bytes_moved = N * (S * (row_bytes + 16) + 16 * D + 16)
        if dense:   # 2D^2 + 7D per leapfrog (Random dense), 2D^2 + 12D (NUTS: E + U-turn dots)
            flops_launch = lf_launch * (2 * D * D + (12 if nuts else 7) * D)
        else:       # 8D per leapfrog + 8D energies per iteration
            flops_launch = lf_launch * 8 * D + N * S * 8 * D
        kern_s = kern_ms / 1e3
        tfl = flops_launch / kern_s / 1e12
        kname = "hmc_nuts_iters" if nuts else ("hmc_random_iters(dense)" if dense else "hmc_random_iters")
        shape = dict(kernel=kname, dim=D, chains_per_gpu=N, iters_per_step=S, window_rows=R,
                     stream_diag=bool(a.stream_diag), rho=a.rho)
        pm = pmc_traffic(shape)
        hbm = {"bound": "hbm", "achieved": bytes_model / kern_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": bytes_model / kern_s / 1e9 / HBM_PEAK_GBS,
               "traffic": None if pm is None else pm["bytes_per_launch"],
               "traffic_source": None if pm is None else pm.get("source"),
               "kernel": kname, "kernel_ms": kern_ms, "bytes_per_launch": bytes_model, "shape": shape,
               "bytes_model": "SURVEY.md §8(d): (24*D + 24) B per chain-iteration x chains x iterations per launch",
               "bytes_moved_per_launch": bytes_moved,
               "frac_moved": bytes_moved / kern_s / 1e9 / HBM_PEAK_GBS}
        mfma = {"bound": "mfma" if dense else "fp64 vector", "achieved": tfl, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": tfl / FP64_PEAK_TFLOPS,
                "traffic": None if pm is None else pm["bytes_per_launch"], "shape": shape, "kernel": kname,
                "kernel_ms": kern_ms, "flops_per_launch": flops_launch}
        tdesc = f"rho={a.rho} dense-precision MVN" if a.rho != 0 else "unit MVN"
        samp = f"NUTS d_max={a.d_max} (overflow counted, not aborted)" if nuts else "Random-L HMC, L~U{5..19}"
        store_desc = (f"every q_chain row, E, dE stored (circular window of {R} rows)" if store else
                      "rows fed to streaming diagnostics" if sd is not None else "no q_chain rows (ablation)")
        line = {
            "metric": "leapfrog steps/sec (whole node) + ESS/sec, D=100 MVN at 1M chains",
            "value": value,
            "unit": "leapfrog steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": t_max / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (D={D} {tdesc}, starts ~ N(0, 2I), Philox4x32-10 draws)",
            "config": {"workload": f"{samp}, D={D} {tdesc}, dt={a.dt}, {a.chains} chains in total "
                                   f"({N} on rank 0), {S} iterations per step (one fused launch), "
                                   f"{store_desc}, fp_mode={a.fp_mode}",
                       "chains_total": a.chains, "chains_per_gpu": N, "dim": D, "iters_per_step": S,
                       "window_rows": R, "parallelism": f"chains{world}"},
            "roofline": mfma if dense else hbm,
            "compute" if not dense else "memory": mfma if not dense else hbm,
            "accept_rate": None if nuts else acc_all / (a.chains * K * S),
            "leapfrog_per_iteration": lf_all / (a.chains * K * S),
            "lane_utilisation": (lf_local / (16.0 * wave_steps)) if nuts and wave_steps else None,
            "dmax_fraction": (dmax_all / (a.chains * K * S)) if nuts else None,
            "debug_env_unset": True,
            "ess": ess,
        }
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(D, a.cpu_seconds, a.rho, a.sampler, a.d_max)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
