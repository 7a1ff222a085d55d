"""bench.py host logic on CPU: the --gpus N launcher, chain sharding and the q_chain window."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_shard_covers_all_chains_contiguously():
    for total, world in ((1 << 20, 8), (1 << 20, 3), (10, 4), (5, 8)):
        rng = [bench.shard(total, world, r) for r in range(world)]
        assert sum(c for _, c in rng) == total
        off = 0
        for o, c in rng:
            assert o == off
            off += c
        assert max(c for _, c in rng) - min(c for _, c in rng) <= 1


def test_window_rows_divides_timed_rows():
    assert bench.window_rows(800, 125) == 100
    assert bench.window_rows(800, 1000) == 800
    assert bench.window_rows(7 * 40, 100) == 70
    for total in (40, 200, 800, 97):
        for budget in (1, 13, 64, 125):
            r = bench.window_rows(total, budget)
            assert total % r == 0 and r <= max(budget, 1)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_flag_launches_ranks(n):
    """`bench.py --gpus N` without WORLD_SIZE starts N ranks itself (torch.distributed.run as a
    child process) and rank 0 reports n_gpus = N with the chains split by global id."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run",
                          "--chains", "1048576"], capture_output=True, text=True, env=env, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out.stdout
    rep = json.loads(line[0])
    assert rep["n_gpus"] == n
    shards = sorted(rep["shards"])
    assert [s[0] for s in shards] == list(range(n))
    assert sum(s[2] for s in shards) == 1048576
    assert shards[0][1] == 0 and all(shards[i][1] + shards[i][2] == shards[i + 1][1] for i in range(n - 1))


def test_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                         capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_debug_env_refused():
    env = dict(os.environ, HMC_DEBUG_ABLATE="64")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], capture_output=True,
                         text=True, env=env, timeout=120)
    assert out.returncode != 0 and "HMC_DEBUG_ABLATE" in out.stderr


def test_presets_resolve_baseline_configs():
    """--config picks the BASELINE.json shapes; explicit flags still override the preset."""
    a = bench.parse(["--config", "c3"])
    assert (a.chains, a.dim, a.rho, a.sampler) == (262144, 100, 0.95, "random")
    a = bench.parse(["--config", "c5", "--steps", "7"])
    assert (a.chains, a.rho, a.sampler, a.steps, a.warmup) == (65536, 0.95, "nuts", 7, 1)
    a = bench.parse(["--config", "c4"])
    assert a.stream_diag and a.dim == 1000
    assert bench.resolve_chains(a, 8) == (1048576, True)      # c4: 1,048,576 chains on 8 GPUs
    assert bench.resolve_chains(a, 1) == (131072, True)
    a = bench.parse([])
    assert bench.resolve_chains(a, 8) == (1048576, False)     # the metric: 1M chains at any N
    a = bench.parse(["--config", "c1"])
    assert (a.chains, a.dim, a.iters_per_step * a.warmup, a.iters_per_step * a.steps) == (10, 2, 1000, 1000)


def test_c4_dry_run_prints_eight_shards():
    """The c4 job as 8 ranks: 131,072 chains x D=1000 each, 1,048,576 in total."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c4", "--gpus", "8",
                          "--dry-run"], capture_output=True, text=True, env=env, timeout=400)
    assert out.returncode == 0, out.stderr[-2000:]
    rep = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert rep["n_gpus"] == 8 and rep["chains_total"] == 1048576 and rep["scaling"] == "weak"
    assert rep["dim"] == 1000
    shards = sorted(rep["shards"])
    assert [s[1] for s in shards] == [131072 * r for r in range(8)]
    assert all(s[2] == 131072 for s in shards)
