"""sb_train's training-loop hooks on the device-resident trainer (quadswarm_amd.callbacks, PPOTrainer.learn /
save / load):

* DeviceCurriculum (qs_curriculum_step, one HIP launch per env step) against a host restatement of the reference's
  CurriculumCallback._on_step (swarm_rl/custom_callbacks.py:441-468) fed with the same per-step reset_infos: the
  window, window_i, success rate, radius and number of reductions agree exactly (fp64), and every env's capture
  radius on the device is the reduced one;
* qs_curriculum_step_all (the data-parallel form: every rank runs it over all ranks' gathered reset_info rows) over
  this handle's rows concatenated with a second, synthetic rank's: the same host restatement over the concatenation,
  and the radius lands in this handle's envs only;
* a checkpoint written by CheckpointCallback after one iteration, loaded into a fresh trainer (different weights
  and env seed), reproduces the following iteration bitwise: weights, Adam state, env snapshot, rollout buffer
  and the curriculum's device state;
* EvalCallback: the evaluation statistics equal SB3's evaluate_policy / EvalCallback._on_step restated over the eval
  env's recorded per-step rewards and dones (episode rewards and lengths, mean reward, best-model checkpoint on
  improvement only), the curriculum's radius reaches the eval env, and the evaluation episodes are deterministic."""
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
    """CurriculumCallback._on_step (custom_callbacks.py:449-468) restated on the host (oracle/curriculum_oracle.py),
    minus logging / eval env."""
    from curriculum_oracle import CurriculumOracle
    o = CurriculumOracle(r0, sr_thr, decay, W)
    for resets in steps:
        o.step(resets)
    return dict(past=o.past, window_i=o.window_i, success_rate=o.success_rate, radius=o.radius,
                n_shrinks=len(o.history))


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


def test_curriculum_step_all_over_gathered_rows():
    """The kernel over [this handle's reset_info | a synthetic second rank's row] (what the all-gather hands it)."""
    import ctypes
    from curriculum_oracle import CurriculumOracle
    cfg = QuadSwarmConfig.sb_train(num_envs=64, num_agents=4, initial_capture_radius=3.0, seed=5)
    env = QuadSwarmEnv(cfg)
    env.reset()
    env.set_capture_radius(3.0)
    c = NAT.QsCurriculum()
    NAT.check(NAT.lib().qs_curriculum_init(ctypes.byref(c), 3.0, 0.45, 0.9, 40), "init")
    dev = torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8).cuda()
    o = CurriculumOracle(3.0, 0.45, 0.9, 40)
    g = torch.Generator(device="cuda").manual_seed(2)
    other_g = np.random.default_rng(7)
    allr = torch.empty(2 * env.E, dtype=torch.uint8, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    resets = 0
    for t in range(300):
        a = (torch.rand(env.I, 2, device="cuda", generator=g) * 2 - 1).contiguous()
        env.step(a)
        other = other_g.choice([0, 0, 0, 0, 0, 1, 2, 2], size=env.E).astype(np.uint8)   # rank 1: mostly successes
        allr[:env.E].copy_(env.reset_info)
        allr[env.E:].copy_(torch.from_numpy(other))
        NAT.check(NAT.lib().qs_curriculum_step_all(env._h, ctypes.c_void_p(allr.data_ptr()), 2 * env.E,
                                                   ctypes.c_void_p(dev.data_ptr()), st), "step_all")
        row = allr.cpu().numpy()
        resets += int((row != 0).sum())
        o.step(row.tolist())
    got = NAT.QsCurriculum.from_buffer_copy(bytes(dev.cpu().numpy().tobytes()))
    assert resets > 200 and len(o.history) >= 2
    assert got.n_shrinks == len(o.history) and got.window_i == o.window_i
    assert got.radius == o.radius and got.success_rate == o.success_rate
    assert list(got.past)[:40] == list(o.past)
    assert (env.env_f[NAT.ENVF_CAPTURE].cpu().numpy() == np.float32(o.radius)).all()
    with pytest.raises(NAT.QuadSwarmError):      # fewer rows than the handle's own envs
        NAT.check(NAT.lib().qs_curriculum_step_all(env._h, ctypes.c_void_p(allr.data_ptr()), env.E - 1,
                                                   ctypes.c_void_p(dev.data_ptr()), st), "step_all")
    env.close()


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


class RecordingEnv:
    """The eval env with every step's rewards, dones and reset_info recorded (host copies)."""

    def __init__(self, env):
        self.env, self.rec = env, []
        self.I, self.N, self.E, self.cfg = env.I, env.N, env.E, env.cfg

    @property
    def reset_info(self):
        return self.env.reset_info

    def set_capture_radius(self, v):
        self.env.set_capture_radius(v)

    def reset(self):
        self.rec.append("reset")
        return self.env.reset()

    def step(self, a):
        out = self.env.step(a)
        self.rec.append((out[1].double().cpu().numpy(), out[2].cpu().numpy().astype(bool),
                         self.env.reset_info.cpu().numpy().copy()))
        return out


def reference_evaluate(rec, n_rows, n_eval_episodes):
    """stable_baselines3 evaluate_policy(return_episode_rewards=True) restated over a recorded run (one evaluation:
    the steps after its reset), per its published algorithm."""
    targets = np.array([(n_eval_episodes + i) // n_rows for i in range(n_rows)])
    counts = np.zeros(n_rows, dtype=int)
    cr, cl = np.zeros(n_rows), np.zeros(n_rows, dtype=int)
    er, el = [], []
    for r, d, _ in rec:
        cr += r
        cl += 1
        for i in range(n_rows):
            if counts[i] < targets[i] and d[i]:
                er.append(cr[i])
                el.append(cl[i])
                counts[i] += 1
                cr[i] = 0
                cl[i] = 0
        if not (counts < targets).any():
            break
    return er, el


def test_eval_callback_matches_sb3_evaluate_policy(tmp_path):
    from quadswarm_amd.callbacks import EvalCallback
    cfg, env, pol, tr = make(seed=4, E=64, n_steps=16, radius=3.0)
    ecfg = QuadSwarmConfig.sb_train(num_envs=1, num_agents=4, initial_capture_radius=3.0, seed=99)
    eenv = RecordingEnv(QuadSwarmEnv(ecfg))
    cur = DeviceCurriculum(0.5, 0.9, 3.0, verbose=0, eval_env=eenv, eval_freq=0)   # pushes its radius only
    ev = EvalCallback(eenv, n_eval_episodes=6, eval_freq=16, log_path=str(tmp_path / "eval"),
                      best_model_save_path=str(tmp_path / "best"), verbose=0)
    bests = []

    class Watch(TrainerCallback):
        def on_iteration_end(self, trainer):
            bests.append((ev.last_mean_reward, ev.best_mean_reward, len(ev.best_saved)))
    tr.learn(3 * 16 * env.I, callback=[cur, ev, Watch()])
    # three evaluations, each: a reset, then steps until every row met its target
    runs, curr = [], None
    for x in eenv.rec:
        if isinstance(x, str):
            curr = []
            runs.append(curr)
        else:
            curr.append(x)
    assert len(runs) == 3
    res = np.load(str(tmp_path / "eval" / "evaluations.npz"))
    assert list(res["timesteps"]) == [16 * env.I * k for k in (1, 2, 3)]
    best, nbest = -np.inf, 0
    for k, run in enumerate(runs):
        er, el = reference_evaluate(run, eenv.I, 6)
        assert len(er) == 6                      # targets (6 + i) // 4 = [1, 1, 2, 2]
        assert list(res["results"][k]) == er and list(res["ep_lengths"][k]) == el
        m = float(np.mean(er))
        assert bests[k][0] == m
        if m > best:
            best, nbest = m, nbest + 1
        assert bests[k][1] == best and bests[k][2] == nbest
    assert nbest >= 1 and os.path.exists(str(tmp_path / "best" / "best_model.pt"))
    # the curriculum's radius (shrunk or not) is the eval env's
    assert (eenv.env.env_f[NAT.ENVF_CAPTURE].cpu().numpy() == np.float32(cur.capture_radius)).all()
    # deterministic policy: re-running an evaluation from the same env state gives the same episodes
    from quadswarm_amd.callbacks import evaluate_policy
    s0 = eenv.env.get_state()
    a = evaluate_policy(tr.policy, eenv, 6)
    eenv.env.set_state(s0)
    b = evaluate_policy(tr.policy, eenv, 6)
    assert a == b
    env.close()
    eenv.env.close()
