"""bench.py's multi-rank path on the GPU: the N-rank job is the 1-rank job.

Chains shard by global id, and Philox draws and start points are keyed by that id, so a 2-rank run
(torch.distributed.run, gloo process group, both ranks on cuda:0 of a one-GPU box) must integrate
exactly the same leapfrogs, accept exactly the same proposals and, through the all-reduced
split-chain statistics (diagnostics.combine via the group), give the same R-hat / ESS as the
1-rank run of the same total chains (samplers.py:410 is the chain loop the
sharding replaces)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(args, n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--no-cpu-baseline", "--no-telemetry",
           "--chain-budget-gb", "1"] + args + (["--backend", "gloo"] if n > 1 else [])
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("args", [
    ["--chains", "3000", "--steps", "2", "--warmup", "1", "--iters-per-step", "10"],
    ["--chains", "1000", "--dim", "200", "--stream-diag", "--steps", "3", "--warmup", "1", "--iters-per-step", "8"],
    ["--config", "c5", "--chains", "700", "--steps", "1", "--warmup", "1", "--iters-per-step", "4"],
], ids=["unit-d100", "stream-d200", "nuts"])
def test_two_ranks_equal_one_rank(args):
    one = _bench(args, 1)
    two = _bench(args, 2)
    assert two["n_gpus"] == 2 and two["config"]["chains_total"] == one["config"]["chains_total"]
    assert two["leapfrogs"] == one["leapfrogs"] > 0
    assert two["accepts"] == one["accepts"]
    if one["dmax_fraction"] is not None:
        assert two["dmax_fraction"] == one["dmax_fraction"]
    for k in ("rhat_median", "rhat_max", "n_eff_median", "n_eff_min"):
        assert two["ess"][k] == pytest.approx(one["ess"][k], rel=1e-10), k
    assert two["ess"]["samples_per_chain"] == one["ess"]["samples_per_chain"]
