"""world_size-2 gloo tests of the data-parallel PPO update: one all_reduce of the flat
gradient bucket per minibatch averages the ranks' gradients, and the ranks' weights stay identical
through a full PPO iteration although each rank collects its own shard of experience.
CPU stand-in env + oracle GAE (the product GAE is the HIP kernel)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_ppo_cpu import ToyEnv, gae_oracle_torch, sb_cfg
from quadswarm_amd.ppo import FlatGradBucket, PPOConfig, PPOTrainer, SwarmActorCritic


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)          # different init per rank: the trainer must broadcast rank 0's
    _, pc = sb_cfg(rnn_num_layers=2, rnn_size=32, neighbor_hidden_size=16)
    pol = SwarmActorCritic(pc)
    env = ToyEnv(I=16, seed=rank)          # each rank its own shard of experience
    tr = PPOTrainer(env, pol, PPOConfig(n_steps=8, batch_size=32, n_epochs=2), device="cpu",
                    gae_fn=gae_oracle_torch, seed=7)
    # (1) bucket all-reduce = mean of the ranks' local gradients
    obs = torch.randn(8, 28, generator=torch.Generator().manual_seed(rank))
    act = torch.rand(8, 2, generator=torch.Generator().manual_seed(50 + rank)) * 1.6 - 0.8
    tr.bucket.zero()
    v, lp, _ = pol.evaluate_actions(obs, act)
    (v.square().mean() - lp.mean()).backward()
    local = tr.bucket.flat.clone()
    tr.bucket.all_reduce_mean()
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    mean_err = float((torch.stack(allg).mean(0) - tr.bucket.flat).abs().max())
    # (2) a PPO iteration keeps the replicas identical
    tr.learn_iteration()
    w = torch.cat([p.detach().flatten() for p in pol.parameters()])
    ws = [torch.empty_like(w) for _ in range(world)]
    dist.all_gather(ws, w)
    if rank == 0:
        q.put((mean_err, float((ws[0] - ws[1]).abs().max()), tr.num_timesteps))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_ppo_update_stays_in_lockstep():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    mean_err, wdiff, steps = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mean_err < 1e-7
    assert wdiff == 0.0
    assert steps == 8 * 16 * 2          # global num_timesteps: both ranks' agents


def test_bucket_without_process_group_is_identity():
    pol = SwarmActorCritic(sb_cfg(rnn_num_layers=1, rnn_size=16, neighbor_hidden_size=8)[1])
    b = FlatGradBucket(pol.parameters())
    b.flat.normal_()
    before = b.flat.clone()
    b.all_reduce_mean()
    assert torch.equal(before, b.flat)
    assert np.isfinite(float(b.clip_norm_(0.5)))
