"""BASELINE config 5 on the GPU: the per-GPU shard of the 32-drone x 8192-env run over 8 MI355X
(1024 envs x 32 drones per GPU, pos_vel k = 6, specialised kernels), and the data-parallel pieces the
8-GPU run uses -- env shards keyed by drone_id_offset, and the RCCL all-reduce of the flat PPO gradient
bucket (world size 1 here: the 8-GPU run is the driver's).

The full-size episode is checked through size-independent properties (the oracle comparisons at N = 32
live in test_gpu_parity.py at 64 envs): the episode boundary at tick 1501, finiteness, the obs clip
boxes, the static_same_goal spawn box at rest, and bitwise shard invariance."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def c5(**over):
    kw = dict(num_envs=1024, num_agents=32, neighbor_visible_num=6, neighbor_obs_type="pos_vel", seed=0)
    kw.update(over)
    return QuadSwarmConfig(**kw)


def test_c5_full_size_episode():
    cfg = c5()
    env = QuadSwarmEnv(cfg)
    assert env.specialized
    I = 1024 * 32
    obs = env.reset()
    assert obs.shape == (I, 18 + 6 * 6)
    a = torch.empty(I, 4, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    n_done = 0
    for t in range(cfg.ep_len + 3):
        a.uniform_(-1, 1, generator=g)
        obs, rew, done, term = env.step(a)
        if done.any():
            assert bool(done.all())      # synchronised episodes end together
            assert t == cfg.ep_len       # tick > ep_len: the 1501st step
            assert torch.isfinite(term).all()
            n_done += 1
            f = env.drone_fields()
            pos = f["pos"]
            assert (pos[:, 0:2].abs() <= 2.0 + 1e-5).all() and (pos[:, 2] >= 0.75 - 1e-6).all()
            assert (pos[:, 2] <= 4.0 + 1e-5).all() and (f["vel"] == 0).all() and (f["omega"] == 0).all()
            assert (env.env_state[0] == 0).all()
        if t % 100 == 0 or done.any():
            assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
            nb = obs[:, 18:].view(-1, 6, 6)
            assert (nb[:, :, 0:3].abs() <= 10.0).all() and (nb[:, :, 3:6].abs() <= 6.0).all()
            assert (obs[:, 6:15].abs() <= 1.0 + 1e-3).all()
    assert n_done == 1
    assert env.counters() == {"nonfinite_obs": 0, "nonfinite_rew": 0, "nonfinite_state": 0}


def test_c5_shards_equal_one_handle():
    """Two 512-env shards (the second keyed from drone 512 * 32) == the 1024-env handle, bitwise."""
    big = QuadSwarmEnv(c5(episode_duration=0.3))
    s0 = QuadSwarmEnv(c5(num_envs=512, episode_duration=0.3))
    s1 = QuadSwarmEnv(c5(num_envs=512, episode_duration=0.3, drone_id_offset=512 * 32))
    ob = big.reset().clone()
    assert torch.equal(torch.cat([s0.reset(), s1.reset()]), ob)
    g = torch.Generator(device="cuda").manual_seed(2)
    half = 512 * 32
    for t in range(70):          # two episode ends (30-tick episodes) with fused resets
        act = (torch.rand(1024 * 32, 4, device="cuda", generator=g) * 2 - 1).contiguous()
        r = [x.clone() for x in big.step(act)]
        p = [x.clone() for x in s0.step(act[:half].contiguous())]
        q = [x.clone() for x in s1.step(act[half:].contiguous())]
        for x, y, z in zip(r, p, q):
            assert torch.equal(torch.cat([y, z]), x), t
    assert torch.equal(torch.cat([s0.state, s1.state], 1), big.state)


_RCCL_CHILD = r"""
import json, os, sys
sys.path[:0] = [os.path.join(os.environ["QS_ROOT"], "quad-swarm-rl-stable-baselines3_amd")]
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))   # RCCL first, before other GPU work
from quadswarm_amd import QuadSwarmConfig
from quadswarm_amd.env import QuadSwarmEnv
from quadswarm_amd.ppo import PolicyConfig, PPOConfig, PPOTrainer, SwarmActorCritic
torch.manual_seed(0)
cfg = QuadSwarmConfig(num_envs=64, num_agents=32, neighbor_visible_num=6, seed=1, episode_duration=0.1)
env = QuadSwarmEnv(cfg)
pol = SwarmActorCritic(PolicyConfig.for_env(cfg, rnn_size=64, neighbor_hidden_size=64)).cuda()
tr = PPOTrainer(env, pol, PPOConfig(n_steps=16, batch_size=4096, n_epochs=1), seed=0)
# the flat gradient bucket through RCCL: world size 1, so the sum is the bucket itself
tr.bucket.flat.copy_(torch.randn(tr.bucket.flat.numel(), device="cuda", generator=torch.Generator("cuda").manual_seed(3)))
before = tr.bucket.flat.clone()
dist.all_reduce(tr.bucket.flat)
roundtrip = bool(torch.equal(before, tr.bucket.flat))
tr.bucket.all_reduce_mean()
stats = tr.learn_iteration()
finite = all(bool(torch.isfinite(p).all()) for p in pol.parameters())
t = torch.tensor([1.0], device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(), "roundtrip": roundtrip,
                  "finite": finite, "bound": tr.bucket.check_bound(), "n_updates": stats["n_updates"],
                  "max": float(t.item()), "params": tr.bucket.flat.numel()}))
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_bucket_allreduce_and_ppo_iteration():
    """A child process (RCCL initialised before any other GPU call, as bench.py's N > 1 path does) runs the
    flat-bucket all-reduce over RCCL and one PPO iteration on a 32-drone HIP env."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", QS_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _RCCL_CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["roundtrip"] and out["finite"] and out["bound"]
    assert out["n_updates"] == 16 * 64 * 32 // 4096 and out["max"] == 1.0
