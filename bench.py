"""Benchmark: leapfrog steps/s (whole job) + ESS/s of the many-chain Random-trajectory HMC
on a D=100 unit-MVN target (BASELINE.json metric; configs[1] shape), fp64.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

One step = ONE kernel launch of hmc_random_iters that advances every chain of this GPU by
--iters-per-step HMC iterations (auto: 40, or fewer when the stored q_chain would exceed
--chain-budget-gb; HMC_sampler.gen_sample itself fuses a whole run into one launch) (momentum resample, L ~ U{5..19} leapfrogs, Metropolis test,
sample stored).  Chains shard over GPUs by global chain id (Philox keyed by it): weak scaling,
no data-path collective; RCCL is used only for the diagnostics all-reduce after timing.
Rank 0 prints one JSON line.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "understanding-hmc_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector = FP64 matrix peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chains", type=int, default=131072, help="chains per GPU (8 GPUs -> 1,048,576)")
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--iters-per-step", type=int, default=0,
                    help="HMC iterations fused into one launch (= one timed step); 0 = auto: 40 for the "
                         "Random sampler (HMC_sampler.gen_sample fuses the whole run into one launch; "
                         "shorter launches pay a per-wave start-up), lowered so the stored q_chain stays "
                         "within --chain-budget-gb; 2 for NUTS")
    ap.add_argument("--chain-budget-gb", type=float, default=100.0,
                    help="HBM budget for the stored q_chain of the timed iterations (auto iters-per-step)")
    ap.add_argument("--fp-mode", default="fast", choices=["fast", "exact"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dt", type=float, default=0.1)
    ap.add_argument("--rho", type=float, default=0.0, help="MVN correlation (0: unit/diagonal kernel; "
                    ">0: dense precision, MFMA kernel, BASELINE config 3 uses 0.95 with 262144 chains)")
    ap.add_argument("--sampler", default="random", choices=["random", "nuts"],
                    help="nuts: BASELINE config 5 (use with --rho 0.95 --chains 65536 --iters-per-step 2)")
    ap.add_argument("--d-max", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget per process")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ess", action="store_true")
    ap.add_argument("--stream-diag", action="store_true",
                    help="no q_chain storage: R-hat/ESS from windowed streaming statistics inside the timed "
                         "loop (config 4: D=1000 at 131072 chains/GPU)")
    ap.add_argument("--tmax", type=int, default=16, help="streaming variogram lags")
    ap.add_argument("--stream-feed", type=int, default=0,
                    help="--stream-diag: steps between diagnostics updates (window of tmax + "
                         "(feed+1)*iters_per_step rows; larger = less variogram carry re-reading); "
                         "0 = auto: every ~60 iterations")
    ap.add_argument("--no-order-tiles", action="store_true",
                    help="dense targets: MFMA tiles in chain order (several iterations per launch) instead of "
                         "L-ordered tiles (one launch per iteration, chains sorted by trajectory length)")
    return ap.parse_args()


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


def cpu_baseline(D, budget, rho=0.0, sampler="random", d_max=10):
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    procs = max(1, min(cores, 16))
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
                sample=f"oracle/hmc_oracle.py {sampler} engine (reference-equivalent NumPy: eigh logpdf per E, "
                       f"SVD mvn per draw), D={D} rho={rho}, {procs} procs x 1 chain x ~{budget:.0f} s, "
                       f"{lf} leapfrogs")


# ------------------------------------------------------------------ profile-derived HBM traffic
def pmc_traffic():
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (profiles/), if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from hmc_amd.engine import NutsEngine, RandomEngine
    from hmc_amd.target import MVNTarget
    from hmc_amd import _lib as H
    from hmc_amd.diagnostics import StreamingDiagnostics, convergence_stats

    D, N, S = a.dim, a.chains, a.iters_per_step
    if S <= 0:
        if a.sampler == "nuts":
            S = 2
        else:
            rows = int(a.chain_budget_gb * 1e9 // (8.0 * N * D))          # q_chain rows that fit the budget
            if a.stream_diag:     # the circular window holds tmax + (feed + 1) * S rows
                S = 20
            elif a.no_ess:
                S = 40
            else:
                S = max(1, min(40, (rows - 1) // max(1, a.warmup + a.steps)))
    W, K = a.warmup, a.steps
    feed_steps = a.stream_feed if a.stream_feed > 0 else max(1, 60 // S)
    n_iter = (W + K) * S
    wu = W * S + 1                     # q_chain rows 0..K*S hold exactly the timed iterations
    cov = np.eye(D) if a.rho == 0 else (np.diag(np.ones(D)) * (1 - a.rho) + a.rho)
    tgt = MVNTarget(np.zeros(D), cov)
    nuts = a.sampler == "nuts"
    if nuts:
        eng = NutsEngine(tgt, N, n_iter, wu, 1, a.d_max, a.dt, rng="philox", seed=a.seed, fp_mode=a.fp_mode,
                         chain_offset=rank * N, store_chain=not a.no_ess, on_dmax="break", device=dev)
    else:
        eng = RandomEngine(tgt, N, n_iter, wu, 1, 5, 20, a.dt, rng="philox", seed=a.seed, fp_mode=a.fp_mode,
                           chain_offset=rank * N, store_chain=not (a.no_ess or a.stream_diag), device=dev,
                           order_tiles=not a.no_order_tiles)
    sd = StreamingDiagnostics(N, D, eng.L_chain - 1, tmax=a.tmax, device=dev) if a.stream_diag else None
    rs = np.random.RandomState(a.seed + rank)
    eng.init(torch.as_tensor(rs.standard_normal((N, D)) * np.sqrt(2.0), device=dev))
    it = 1
    def step(i0, evs=None):
        if sd is not None:
            eng.run_streaming(sd, i0, i0 + S, S, events=evs, feed=S * feed_steps)
        else:
            if evs is not None:
                evs[0].record(stream)
            eng.run(i0, i0 + S)
            if evs is not None:
                evs[1].record(stream)

    stream = torch.cuda.current_stream(dev)
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
    wave_steps = int(c1[H.CNT_LEAPFROG_SQ] - c0[H.CNT_LEAPFROG_SQ])   # NUTS: steps of 16-chain waves
    tot = torch.tensor([float(lf_local), float(acc), elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        s = tot[:2].clone()
        dist.all_reduce(s)
        m = tot[2:].clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot = torch.cat([s, m])
    lf_all, acc_all, t_max, kern_max = tot.cpu().numpy().tolist()
    value = lf_all / t_max
    ess = None
    if not a.no_ess:
        grp = dist.group.WORLD if world > 1 else None
        if sd is not None:
            R, neff = sd.finish(grp)
        else:
            R, neff = convergence_stats(eng.q_chain[:, 1:, :], warm_up_num=0, thin_rate=1, group=grp)
        ess = dict(ess_per_s_median=float(np.median(neff)) / t_max, ess_per_s_min=float(np.min(neff)) / t_max,
                   n_eff_median=float(np.median(neff)), rhat_median=float(np.median(R)),
                   samples_per_chain=K * S,
                   method=(f"streaming windows (tmax={a.tmax}) inside the timed loop" if sd is not None
                           else "stored q_chain, after the timed loop"))

    if rank == 0:
        # algorithmic bytes of one launch (S iterations): per chain-iteration one q_chain row +
        # E + dE (8D + 16 B); per launch q and E_prev are read and written once (16D + 16 B)
        row_bytes = 8 * D if (eng.q_chain is not None or sd is not None) else 0
        bytes_launch = N * (S * (row_bytes + 16) + 16 * D + 16)
        lf_launch = lf_local / K
        dense = a.rho != 0 or nuts
        if dense:   # 2D^2 + 7D per leapfrog (Random dense), 2D^2 + 12D (NUTS: E + U-turn dots)
            flops_launch = lf_launch * (2 * D * D + (12 if nuts else 7) * D)
        else:       # 8D per leapfrog + 8D energies per iteration
            flops_launch = lf_launch * 8 * D + N * S * 8 * D
        kern_s = kern_ms / 1e3
        gbs = bytes_launch / kern_s / 1e9
        tfl = flops_launch / kern_s / 1e12
        traffic = pmc_traffic() if not dense and not nuts else None
        kname = "hmc_nuts_iters" if nuts else ("hmc_random_iters(dense)" if dense else "hmc_random_iters")
        hbm = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
               "traffic": None if traffic is None else traffic.get("bytes_per_launch"),
               "kernel": kname, "kernel_ms": kern_ms, "bytes_per_launch": bytes_launch}
        mfma = {"bound": "mfma" if dense else "fp64 vector", "achieved": tfl, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": tfl / FP64_PEAK_TFLOPS, "traffic": None, "kernel": kname,
                "kernel_ms": kern_ms, "flops_per_launch": flops_launch}
        tdesc = f"rho={a.rho} dense-precision MVN" if a.rho != 0 else "unit MVN"
        samp = f"NUTS d_max={a.d_max} (overflow counted, not aborted)" if nuts else "Random-L HMC, L~U{5..19}"
        line = {
            "metric": "leapfrog steps/sec (whole node) + ESS/sec, D=100 MVN at 1M chains",
            "value": value,
            "unit": "leapfrog steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": t_max / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (D={D} {tdesc}, starts ~ N(0, 2I), Philox4x32-10 draws)",
            "config": {"workload": f"{samp}, D={D} {tdesc}, dt={a.dt}, {N} chains/GPU "
                                   f"({N * world} total), {S} iterations per step (one fused launch), "
                                   f"fp_mode={a.fp_mode}",
                       "chains_per_gpu": N, "dim": D, "iters_per_step": S, "parallelism": f"chains{world}"},
            "roofline": mfma if dense else hbm,
            "compute" if not dense else "memory": mfma if not dense else hbm,
            "accept_rate": None if nuts else acc_all / (N * world * K * S),
            "leapfrog_per_iteration": lf_all / (N * world * K * S),
            "lane_utilisation": (lf_local / (16.0 * wave_steps)) if nuts and wave_steps else None,
            "ess": ess,
        }
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(D, a.cpu_seconds, a.rho, a.sampler, a.d_max)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
