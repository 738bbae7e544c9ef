"""sb_train's training-loop hooks on the device-resident trainer (quadswarm_amd.callbacks, PPOTrainer.learn /
save / load):

* DeviceCurriculum (qs_curriculum_step, one HIP launch per env step) against a host restatement of the reference's
  CurriculumCallback._on_step (swarm_rl/custom_callbacks.py:441-468) fed with the same per-step reset_infos: the
  window, window_i, success rate, radius and number of reductions agree exactly (fp64), and every env's capture
  radius on the device is the reduced one;
* a checkpoint written by CheckpointCallback after one iteration, loaded into a fresh trainer (different weights
  and env seed), reproduces the following iteration bitwise: weights, Adam state, env snapshot, rollout buffer
  and the curriculum's device state."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from quadswarm_amd import QuadSwarmConfig, _native as NAT  # noqa: E402
from quadswarm_amd.callbacks import CheckpointCallback, DeviceCurriculum, TrainerCallback  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from quadswarm_amd.ppo import PolicyConfig, PPOConfig, PPOTrainer, SwarmActorCritic  # noqa: E402


class RecordResets(TrainerCallback):
    """Keeps every step's reset_infos (the host tuple the reference's callback iterates)."""

    def __init__(self):
        self.steps = []

    def on_step(self, ctx):
        self.steps.append(ctx.reset_infos)
        return True


def reference_curriculum(steps, r0, sr_thr, decay, W=40):
    """CurriculumCallback._on_step (custom_callbacks.py:449-468) restated on the host, minus logging / eval env."""
    past, wi, sr, r, n = np.zeros(W), 0, 0.0, r0, 0
    for resets in steps:
        change = False
        for e in resets:
            if e is not None:
                past[wi % W] = e["success"]
                wi += 1
                change = True
        if change:
            sr = np.sum(past) / W
            if sr > sr_thr:
                r = decay * r
                n += 1
                past = np.zeros(W)
    return dict(past=past, window_i=wi, success_rate=sr, radius=r, n_shrinks=n)


def make(seed=0, E=64, n_steps=32, radius=3.0):
    cfg = QuadSwarmConfig.sb_train(num_envs=E, num_agents=4, initial_capture_radius=radius, seed=seed)
    env = QuadSwarmEnv(cfg)
    torch.manual_seed(seed)
    pol = SwarmActorCritic(PolicyConfig.sb_train(cfg)).cuda()
    tr = PPOTrainer(env, pol, PPOConfig(n_steps=n_steps, batch_size=2048, n_epochs=2), seed=seed)
    return cfg, env, pol, tr


def test_device_curriculum_matches_reference_callback():
    # a large starting radius: captures come quickly, so the window fills with successes and the radius shrinks
    # several times within a few rollouts (sb_train's own values: sr 0.95, decay 0.95; here sr 0.5 to reach the
    # branch with mixed outcomes too)
    cfg, env, pol, tr = make(radius=4.0)
    cur = DeviceCurriculum(capture_radius_sr=0.5, capture_radius_decay=0.9, initial_capture_radius=4.0, verbose=0)
    rec = RecordResets()
    tr.learn(3 * 32 * env.I, callback=[cur, rec])
    c = cur.read()
    want = reference_curriculum(rec.steps, 4.0, 0.5, 0.9)
    assert sum(r is not None for s in rec.steps for r in s) > 100       # many episodes ended
    assert want["n_shrinks"] >= 2, want
    assert c.n_shrinks == want["n_shrinks"] and c.window_i == want["window_i"]
    assert c.radius == want["radius"] and c.success_rate == want["success_rate"]
    assert list(c.past)[:40] == list(want["past"])
    caps = env.env_f[NAT.ENVF_CAPTURE].cpu().numpy()
    assert (caps == np.float32(want["radius"])).all()
    assert cur.records["curriculum/capture_radius"] == want["radius"]


def test_resume_from_checkpoint_reproduces_next_iteration_bitwise(tmp_path):
    n_steps = 16
    cfg, env, pol, tr = make(seed=3, n_steps=n_steps, radius=2.0)
    cur = DeviceCurriculum(0.5, 0.9, 2.0, verbose=0)
    ck = CheckpointCallback(save_freq=n_steps, save_path=str(tmp_path), name_prefix="quad_swarm")
    per_it = n_steps * env.I
    tr.learn(2 * per_it, callback=[cur, ck])
    assert [os.path.basename(p) for p in ck.saved] == [f"quad_swarm_{per_it}_steps.pt", f"quad_swarm_{2 * per_it}_steps.pt"]
    want_params = [p.detach().clone() for p in pol.parameters()]
    want_env = env.get_state()
    want_rew = tr.storage.rewards.clone()
    want_adam = [v.clone() for st in tr.optimizer.state.values() for v in st.values() if torch.is_tensor(v)]
    want_cur = bytes(cur.read())

    # a fresh trainer: other weights, other env seed; then the first checkpoint and one more iteration
    cfg2, env2, pol2, tr2 = make(seed=11, n_steps=n_steps, radius=2.0)
    cur2 = DeviceCurriculum(0.5, 0.9, 2.0, verbose=0)
    ck2 = CheckpointCallback(save_freq=n_steps, save_path=str(tmp_path / "b"), name_prefix="quad_swarm")
    tr2.load(ck.saved[0], callbacks=[cur2, ck2])
    assert tr2.num_timesteps == per_it and tr2.iterations == 1
    tr2.learn(2 * per_it, callback=[cur2, ck2])
    for a, b in zip(want_params, pol2.parameters()):
        assert torch.equal(a, b.detach())
    got_adam = [v for st in tr2.optimizer.state.values() for v in st.values() if torch.is_tensor(v)]
    assert len(got_adam) == len(want_adam) and all(torch.equal(a, b) for a, b in zip(want_adam, got_adam))
    assert env2.get_state() == want_env
    assert torch.equal(tr2.storage.rewards, want_rew)
    assert bytes(cur2.read()) == want_cur
    env.close()
    env2.close()
