"""Diagnostic: first divergence between specialised and generic kernels (per state field)."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "quad-swarm-rl-stable-baselines3_amd"))
import torch
from quadswarm_amd import QuadSwarmConfig, _native as N
from quadswarm_amd.env import QuadSwarmEnv

name = sys.argv[1] if len(sys.argv) > 1 else "a4cam"
mk = {"a4cam": lambda: QuadSwarmConfig.sb_train(num_envs=256, num_agents=4, seed=4, neighbor_visible_num=2, episode_duration=0.6),
      "a8": lambda: QuadSwarmConfig.sb_train(num_envs=256, num_agents=8, seed=4, episode_duration=0.6, initial_capture_radius=1.0),
      "c3": lambda: QuadSwarmConfig(num_envs=512, num_agents=8, neighbor_visible_num=6, episode_duration=0.3, seed=4)}[name]
gen, spc = QuadSwarmEnv(mk()), QuadSwarmEnv(mk())
spc.specialize(True)
gen.reset(); spc.reset()
fields = {k: v for k, v in vars(N).items() if k.startswith("F_") and isinstance(v, int)}
g = torch.Generator(device="cuda").manual_seed(11)
for t in range(10):
    a = (torch.rand(gen.I, gen.act_dim, device="cuda", generator=g) * 2 - 1).contiguous()
    o1 = gen.step(a)[0].clone(); o2 = spc.step(a)[0].clone()
    d = (gen.state - spc.state).abs()
    rows = [(int(r), float(d[r].max())) for r in range(d.shape[0]) if d[r].max() > 0]
    names = {v: k for k, v in fields.items()}
    print(f"step {t}: obs maxdiff {float((o1 - o2).abs().max()):.3g}; state rows differing:",
          [(names.get(r, r), f"{m:.3g}") for r, m in rows][:12])
    if rows:
        r = rows[0][0]
        i = int(d[r].argmax())
        print("   first row", names.get(r, r), "drone", i, float(gen.state[r, i]), float(spc.state[r, i]))
        if t > 2:
            break
