"""PPOTrainer.learn's callback protocol and save/load on CPU (the ToyEnv stand-in of test_ppo_cpu; the GPU
trainer's curriculum and bitwise resume are in test_gpu_trainer.py)."""
import torch

from quadswarm_amd.callbacks import CheckpointCallback, TrainerCallback
from quadswarm_amd.ppo import PPOConfig, PPOTrainer, SwarmActorCritic
from test_ppo_cpu import ToyEnv, gae_oracle_torch, sb_cfg


class Log(TrainerCallback):
    def __init__(self, stop_at=None):
        self.events, self.stop_at = [], stop_at

    def on_training_start(self, tr):
        self.events.append("start")

    def on_rollout_start(self, tr):
        self.events.append("rollout")

    def on_step(self, ctx):
        self.events.append(("step", ctx.batch, ctx.num_timesteps, ctx.t))
        return self.stop_at is None or ctx.batch < self.stop_at

    def on_rollout_end(self, tr):
        self.events.append("rollout_end")

    def on_iteration_end(self, tr):
        self.events.append(("iteration", tr.iterations))

    def on_training_end(self, tr):
        self.events.append("end")


def trainer(seed=0):
    torch.manual_seed(seed)
    _, pc = sb_cfg(rnn_num_layers=2, rnn_size=32, neighbor_hidden_size=16)
    pol = SwarmActorCritic(pc)
    return PPOTrainer(ToyEnv(seed=seed), pol, PPOConfig(n_steps=10, batch_size=64, n_epochs=1), device="cpu",
                      gae_fn=gae_oracle_torch)


def test_learn_hook_order_and_counters():
    tr = trainer()
    log = Log()
    tr.learn(25 * 32, callback=log)           # 3 rollouts of 10 steps reach 960 >= 800 timesteps
    steps = [e for e in log.events if isinstance(e, tuple) and e[0] == "step"]
    assert [s[1] for s in steps] == list(range(1, 31))                  # batch = env steps so far
    assert [s[2] for s in steps] == [32 * b for b in range(1, 31)]      # num_timesteps already advanced (SB3 order)
    assert [s[3] for s in steps[:12]] == list(range(10)) + [0, 1]
    assert log.events[0] == "start" and log.events[-1] == "end"
    assert log.events[1] == "rollout" and log.events[12] == "rollout_end" and log.events[13] == ("iteration", 1)
    assert tr.iterations == 3 and tr.num_timesteps == 960


def test_on_step_false_stops_before_the_update():
    tr = trainer()
    log = Log(stop_at=15)
    w = [p.detach().clone() for p in tr.policy.parameters()]
    tr.learn(10 ** 6, callback=log)
    assert tr.env_steps == 15 and tr.iterations == 1          # the second rollout stopped at its 5th step
    assert ("iteration", 2) not in log.events and log.events[-1] == "end"
    assert any(not torch.equal(a, b) for a, b in zip(w, tr.policy.parameters()))   # the first update ran


def test_checkpoint_callback_and_save_load_round_trip(tmp_path):
    tr = trainer()
    ck = CheckpointCallback(save_freq=10, save_path=str(tmp_path), name_prefix="quad_swarm")
    tr.learn(20 * 32, callback=[ck])
    assert [p.split("/")[-1] for p in ck.saved] == ["quad_swarm_320_steps.pt", "quad_swarm_640_steps.pt"]
    tr2 = trainer(seed=5)
    ck2 = CheckpointCallback(save_freq=10, save_path=str(tmp_path / "b"))
    c = tr2.load(ck.saved[-1], callbacks=[ck2])
    assert c["format"] == PPOTrainer.CKPT_FORMAT
    assert tr2.num_timesteps == 640 and tr2.env_steps == 20 and tr2.iterations == 2 and ck2.n_calls == 20
    for a, b in zip(tr.policy.parameters(), tr2.policy.parameters()):
        assert torch.equal(a, b)
    sa, sb = tr.optimizer.state_dict(), tr2.optimizer.state_dict()
    assert sa["param_groups"] == sb["param_groups"]
    for k in sa["state"]:
        for n, v in sa["state"][k].items():
            assert torch.equal(v, sb["state"][k][n])
    assert torch.equal(tr.gen.get_state(), tr2.gen.get_state())
    assert torch.equal(tr.last_obs, tr2.last_obs) and torch.equal(tr.last_done, tr2.last_done)


def test_reference_state_dict_names_round_trip():
    tr = trainer()
    sd = tr.policy.reference_state_dict()
    assert any(k.startswith("actor_core.core.") for k in sd) and not any(k.startswith("actor_core.0") for k in sd)
    tr2 = trainer(seed=9)
    tr2.policy.load_reference_state_dict(sd)
    for a, b in zip(tr.policy.parameters(), tr2.policy.parameters()):
        assert torch.equal(a, b)
