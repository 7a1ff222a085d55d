"""The N>1 path with the device kernels in the loop, on the one GPU of a test box.

bench.py shards chains by global id (`chain_offset` keys Philox) and the only exchange is the
all-reduce inside hmc_amd.diagnostics (RCCL over xGMI on a node).  A one-GPU box cannot hold a
two-rank RCCL communicator (RCCL refuses two ranks on one device), so:
  * test_rccl_single_rank: a real `nccl` (= RCCL) process group of one rank runs
    convergence_stats(group=...) on device tensors the sampler kernels wrote; it must equal the
    group-less call (the RCCL all-reduce path executes, with the kernels' outputs as its input);
  * test_two_rank_sharded_kernels: two ranks (`gloo`, device tensors) each run the production
    Random kernel on cuda:0 for their half of the chains; the combined R-hat / ESS must equal
    one process sampling all chains (samples are identical per chain: same Philox keys);
  * test_exact_streaming_ranks (round 6): the same with q_chain never stored -- each rank feeds
    its shard's split halves to the exact streaming statistics (hmc_half_sums in the sampler
    loop) and StreamingDiagnostics.finish(group) combines the ranks' sums (shift re-centring +
    all-reduce), over a one-rank RCCL group and over two gloo ranks.
Ranks are spawned processes (at most 2 on the card).  Reference: the serial chain loop
samplers.py:410 that the sharding replaces; utils.py:77-159 for the statistics.
"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

pytestmark = pytest.mark.gpu

N_ALL, D, NITER = 512, 24, 41


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sample(offset, n):
    """Chains offset .. offset + n - 1 of the fixed job: production Random kernel, q_chain on device."""
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    cov = 0.5 * np.eye(D) + 0.5
    eng = RandomEngine(MVNTarget(np.zeros(D), cov), n, NITER, 1, 1, 5, 20, 0.1, rng="philox", seed=7,
                       fp_mode="fast", chain_offset=offset, store_chain=True, device="cuda:0")
    q0 = np.random.RandomState(3).standard_normal((N_ALL, D))[offset:offset + n]
    eng.init(torch.as_tensor(q0, device="cuda:0"))
    eng.run(1, NITER + 1)
    torch.cuda.synchronize()
    return eng.q_chain


def _worker(rank, world, port, backend, out):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "understanding-hmc_amd")]
    from hmc_amd.diagnostics import convergence_stats
    torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        n = N_ALL // world
        qc = _sample(rank * n, n)
        R, neff = convergence_stats(qc[:, 1:, :], thin_rate=1, warm_up_num=0, group=dist.group.WORLD)
        R0, neff0 = convergence_stats(qc[:, 1:, :], thin_rate=1, warm_up_num=0) if world == 1 else (None, None)
        out[rank] = (R, neff, R0, neff0)
    finally:
        dist.destroy_process_group()


def _run(world, backend):
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_worker, args=(world, _free_port(), backend, out), nprocs=world, join=True)
    return dict(out)


def test_rccl_single_rank():
    out = _run(1, "nccl")
    R, neff, R0, neff0 = out[0]
    np.testing.assert_array_equal(R, R0)
    np.testing.assert_array_equal(neff, neff0)
    assert np.all(np.isfinite(R)) and np.all(R > 0.9)


def test_two_rank_sharded_kernels():
    from hmc_amd.diagnostics import convergence_stats
    two = _run(2, "gloo")
    R_all, neff_all = convergence_stats(_sample(0, N_ALL)[:, 1:, :], thin_rate=1, warm_up_num=0)
    for rank in (0, 1):
        R, neff = two[rank][:2]
        np.testing.assert_allclose(R, R_all, rtol=1e-12)
        np.testing.assert_allclose(neff, neff_all, rtol=1e-10)


def _worker_stream(rank, world, port, backend, out):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "understanding-hmc_amd")]
    from hmc_amd.diagnostics import StreamingDiagnostics
    from hmc_amd.engine import RandomEngine
    from hmc_amd.target import MVNTarget
    torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        n = N_ALL // world
        off = rank * n
        cov = 0.5 * np.eye(D) + 0.5
        eng = RandomEngine(MVNTarget(np.zeros(D), cov), n, NITER, 1, 1, 5, 20, 0.1, rng="philox", seed=7,
                           fp_mode="fast", chain_offset=off, store_chain=False, device="cuda:0")
        q0 = np.random.RandomState(3).standard_normal((N_ALL, D))[off:off + n]
        eng.init(torch.as_tensor(q0, device="cuda:0"))
        sd = StreamingDiagnostics(n, D, eng.L_chain - 1, device="cuda:0", mode="exact")
        eng.run_streaming(sd, 1, NITER + 1, 8)
        R, neff = sd.finish(dist.group.WORLD)
        out[rank] = (R, neff, dict(sd.info))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(1, "nccl"), (2, "gloo")])
def test_exact_streaming_ranks(world, backend):
    from hmc_amd.diagnostics import convergence_stats
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_worker_stream, args=(world, _free_port(), backend, out), nprocs=world, join=True)
    R_all, neff_all = convergence_stats(_sample(0, N_ALL)[:, 1:, :], thin_rate=1, warm_up_num=0)
    for rank in range(world):
        R, neff, info = out[rank]
        assert info["mode"] == "streaming-exact" and info["truncated_dims"] == 0
        np.testing.assert_allclose(R, R_all, rtol=1e-10)
        np.testing.assert_allclose(neff, neff_all, rtol=1e-8)
