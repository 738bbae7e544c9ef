"""bench.py's multi-stream layout: one GPU's shard split into S env blocks, each its own handle keyed by
its global drone ids and stepped on its own HIP stream, must produce exactly what the one big handle does
(same obs, rewards, dones, bitwise) — for flavor B, obstacles (C4 preset) and flavor A."""
import pytest
import torch

from quadswarm_amd import QuadSwarmConfig
from quadswarm_amd.env import QuadSwarmEnv

pytestmark = pytest.mark.gpu


def _cfg(kind, E, **over):
    if kind == "c4dr":
        return QuadSwarmConfig.c4(num_envs=E, num_agents=8, seed=5, episode_duration=0.3,
                                  replay_buffer_sample_prob=0.75, domain_random=True, obst_density_random=True,
                                  obst_size_random=True, obst_density_min=0.05, obst_density_max=0.2,
                                  obst_size_min=0.3, obst_size_max=0.6, **over)
    if kind == "c3mixr":
        return QuadSwarmConfig(num_envs=E, num_agents=8, neighbor_visible_num=6, neighbor_obs_type="pos_vel",
                               seed=5, episode_duration=0.3, quads_mode="mix", replay_buffer_sample_prob=0.75,
                               **over)
    if kind == "c4":
        return QuadSwarmConfig.c4(num_envs=E, num_agents=8, seed=5, episode_duration=0.3, **over)
    if kind == "a8":
        return QuadSwarmConfig.sb_train(num_envs=E, num_agents=8, seed=5, episode_duration=0.3, **over)
    return QuadSwarmConfig(num_envs=E, num_agents=8, neighbor_visible_num=6, neighbor_obs_type="pos_vel",
                           seed=5, episode_duration=0.3, **over)


@pytest.mark.parametrize("kind", ["c3", "c4", "a8", "c3mixr", "c4dr"])
def test_stream_blocks_equal_one_handle(kind):
    E, S, N = 128, 4, 8
    big = QuadSwarmEnv(_cfg(kind, E))
    streams = [torch.cuda.Stream() for _ in range(S)]
    blocks = [QuadSwarmEnv(_cfg(kind, E // S, drone_id_offset=s * (E // S) * N)) for s in range(S)]
    ob = big.reset().clone()
    parts = []
    for b, st in zip(blocks, streams):
        with torch.cuda.stream(st):
            parts.append(b.reset().clone())
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts), ob)
    g = torch.Generator(device="cuda").manual_seed(3)
    rows = (E // S) * N
    for t in range(60):
        act = (torch.rand(E * N, big.cfg.act_dim, device="cuda", generator=g) * 2 - 1).contiguous()
        ref = [x.clone() for x in big.step(act)[:3]]
        torch.cuda.synchronize()
        outs = []
        for s, (b, st) in enumerate(zip(blocks, streams)):
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                outs.append([x.clone() for x in b.step(act[s * rows:(s + 1) * rows].contiguous())[:3]])
        torch.cuda.synchronize()
        for i in range(3):
            assert torch.equal(torch.cat([o[i] for o in outs]), ref[i]), (kind, t, i)
