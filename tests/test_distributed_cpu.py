"""world_size-2 gloo tests of the sharded (multi-GPU) path, on CPU.

The env shards across ranks with no data-path collective: each rank owns a contiguous block of
envs and keys its Philox streams with drone_id_offset = rank * drones_per_rank.  Here the CPU
oracle stands in for the per-rank GPU env (same keying), and the test checks that the union of
the shards is exactly the single-process run, and that bench.py's max-over-ranks timing and
agent-step accounting behave under torch.distributed (gloo).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from parity_utils import oracle_params
from quadswarm_amd import QuadSwarmConfig

E_TOTAL, N, STEPS = 16, 8, 30


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_shard(rank, world, e_local, steps, seed=5):
    cfg = QuadSwarmConfig(num_envs=e_local, num_agents=N, episode_duration=0.15, seed=seed)
    p = oracle_params(cfg)
    p.id_offset = rank * e_local * N
    env = O.OracleEnv(p, seed=seed)
    obs = [env.reset()]
    rng = np.random.default_rng(99)
    acts = rng.uniform(-1, 1, (steps, E_TOTAL * N, 4))
    rews = []
    for t in range(steps):
        a = acts[t][rank * e_local * N:(rank + 1) * e_local * N]
        o, r, d, _ = env.step(a, nthreads=1)
        obs.append(o)
        rews.append(r)
    return np.stack(obs), np.stack(rews)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    e_local = E_TOTAL // world
    obs, rews = run_shard(rank, world, e_local, STEPS)
    # gather shards (test-only: the product path has no data-path collective)
    ob = torch.from_numpy(obs)
    gathered = [torch.empty_like(ob) for _ in range(world)]
    dist.all_gather(gathered, ob)
    # bench.py's timing reduction: max over ranks
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((torch.cat(gathered, dim=1).numpy(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, tmax = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want, _ = run_shard(0, 1, E_TOTAL, STEPS)
    np.testing.assert_array_equal(got, want)
    assert tmax == 2.0


def test_shard_offsets_change_streams():
    a, _ = run_shard(0, 2, 4, 2)
    b, _ = run_shard(1, 2, 4, 2)
    assert not np.allclose(a[0], b[0])   # different drones -> different spawns
