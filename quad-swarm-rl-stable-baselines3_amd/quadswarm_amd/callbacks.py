"""sb_train's training-loop hooks on the device-resident trainer (PPOTrainer.learn).

The reference passes SB3 callbacks to `model.learn` (swarm_rl/sb_train.py:70-103): CheckpointCallback
(swarm_rl/custom_callbacks.py:131-208), EvalCallback (:228-427), CurriculumCallback (:429-468, itself an EvalCallback)
and a TensorBoard note.  SB3 calls `callback.on_step()` after every VecEnv step of a rollout, with
`training_env.reset_infos` and `training_env.batch` readable.  Here:

  TrainerCallback   the hook points (on_training_start / on_rollout_start / on_step(ctx) / on_rollout_end /
                    on_iteration_end / on_training_end); on_step returning False stops learn(), like SB3
  StepContext       what on_step sees: the step's device tensors (obs, rewards, dones, actions, reset_info) and,
                    lazily, the reference's host-side `reset_infos` tuple / `batch` (reading reset_infos copies
                    reset_info to the host -- one sync; the device callbacks below never do)
  DeviceCurriculum  CurriculumCallback with its window and radius in device memory: one qs_curriculum_step launch
                    per env step (csrc/qs_curriculum.h), the struct read once per rollout to log and to write the
                    reference's curriculum checkpoints; with an eval env it also runs the EvalCallback the reference's
                    CurriculumCallback inherits (eval_freq 1000, 10 episodes, sb_train.py:86-93)
  EvalCallback      deterministic evaluation episodes on a separate env every eval_freq env steps (SB3's
                    evaluate_policy restated below), evaluations.npz, best-model checkpoint on a new best mean reward
  CheckpointCallback  the reference's periodic checkpoint (every save_freq env steps, named
                    {name_prefix}_{num_timesteps}_steps), written at the end of the iteration in which the period
                    elapsed as a resumable PPOTrainer checkpoint (PPOTrainer.save)

Data-parallel training (one process per GPU, rank r owns a contiguous block of the global envs).  The
reference runs ONE VecEnv, so its callbacks see every env; here:
  * DeviceCurriculum all-gathers every rank's reset_info row after each env step (one small RCCL all_gather, rank-major
    = global env order) and every rank runs the curriculum kernel over the concatenation (qs_curriculum_step_all):
    every rank holds the same window and radius and sets it on its own envs -- one curriculum over all envs, as in
    the reference;
  * num_timesteps counts every rank's agents (PPOTrainer), so save_freq / eval_freq / total_timesteps are global;
  * checkpoints are collective: every rank's env shard is gathered into rank 0's one file (PPOTrainer.save);
  * evaluation runs on rank 0's eval env; its mean reward is broadcast, so every rank takes the same best-model
    decision (and joins the collective save); logs and prints come from rank 0 only.

Differences from the SB3 callbacks (documented, deliberate):
  * checkpoints are written at the rollout / iteration boundary in which the reference would have written them
    mid-rollout.  The policy only changes in the update, so a model saved mid-rollout and at the end of that
    rollout holds the same weights; the iteration boundary is where a trainer checkpoint is resumable.  The
    curriculum's checkpoints (one per radius reduction) are all written at the end of the rollout in which the
    reductions happened (or at the end of training, if learn() stopped mid-rollout): each holds the
    end-of-rollout env state, with the radius that rollout ended with.
  * EvalCallback's success buffer: the reference fills it from `info["is_success"]`, which no env of the reference
    sets, so `eval/success_rate` is never logged there and is not logged here; the capture outcome of the counted
    episodes (the env's reset_infos {"success"}) is logged as `eval/capture_success_rate` (an addition).
"""
import ctypes
import os

import numpy as np
import torch

from . import _native as NAT


def _dist():
    import torch.distributed as dist
    return dist


def _is_main(trainer):
    return getattr(trainer, "rank", 0) == 0


class TrainerCallback:
    """SB3 BaseCallback's hook points for PPOTrainer.learn()."""

    def on_training_start(self, trainer):
        pass

    def on_rollout_start(self, trainer):
        pass

    def on_step(self, ctx) -> bool:
        return True

    def on_rollout_end(self, trainer):
        pass

    def on_iteration_end(self, trainer):
        pass

    def on_training_end(self, trainer):
        pass

    def prepare_eval(self, trainer, eval_env):
        """Called by EvalCallback before it evaluates on eval_env (DeviceCurriculum pushes its radius)."""

    # trainer checkpoints carry every callback's state (PPOTrainer.save / load)
    def state_dict(self):
        return {}

    def load_state_dict(self, sd):
        pass


class StepContext:
    """One env step of a rollout, as on_step sees it (SB3: self.locals + self.training_env).  Device tensors are the
    step's buffers (overwritten by the next step).  Under data parallelism they are this rank's shard."""

    def __init__(self, trainer, t, obs, rewards, dones, actions):
        self.trainer, self.t = trainer, t
        self.obs, self.rewards, self.dones, self.actions = obs, rewards, dones, actions
        self.num_timesteps = trainer.num_timesteps
        self.batch = trainer.env_steps          # SubprocVecEnvCustom.batch: steps taken so far
        env = trainer.env
        self.reset_info = getattr(env, "reset_info", None)   # device u8 [E]: 0 none, 1/2 {"success": False/True}
        self._reset_infos = None

    @property
    def reset_infos(self):
        """The reference's VecEnv.reset_infos for this step: per env {"success": bool} (flavor A) / {} (flavor B)
        for envs the step reset, else None.  Copies the step's reset_info to the host (a sync)."""
        if self._reset_infos is None:
            ri = self.reset_info.cpu().tolist()
            a = getattr(getattr(self.trainer.env, "cfg", None), "flavor", "A") == "A"
            self._reset_infos = tuple(None if v == 0 else ({"success": v == 2} if a else {}) for v in ri)
        return self._reset_infos


def gather_env_rows(trainer, row, buf=None):
    """All ranks' copies of a per-env row (e.g. reset_info u8 [E]), rank-major = global env order: one all_gather.
    Returns `row` itself on a single rank."""
    if not getattr(trainer, "distributed", False):
        return row
    dist = _dist()
    world = trainer.world_size
    if buf is None or buf.numel() != world * row.numel() or buf.device != row.device:
        buf = torch.empty(world * row.numel(), dtype=row.dtype, device=row.device)
    dist.all_gather_into_tensor(buf, row.contiguous(), group=trainer.group)
    return buf


def hip_curriculum_step(trainer, dev_state, reset_all):
    """The curriculum update on the device (csrc/qs_curriculum.h): over this handle's own reset_info
    (qs_curriculum_step) or over every rank's (qs_curriculum_step_all, reset_all = the gathered rows)."""
    env = trainer.env
    st = ctypes.c_void_p(torch.cuda.current_stream(trainer.device).cuda_stream)
    L = NAT.lib()
    if reset_all is None or reset_all is getattr(env, "reset_info", None):
        NAT.check(L.qs_curriculum_step(env._h, ctypes.c_void_p(dev_state.data_ptr()), st), "qs_curriculum_step")
    else:
        NAT.check(L.qs_curriculum_step_all(env._h, ctypes.c_void_p(reset_all.data_ptr()), int(reset_all.numel()),
                                           ctypes.c_void_p(dev_state.data_ptr()), st), "qs_curriculum_step_all")


class DeviceCurriculum(TrainerCallback):
    """CurriculumCallback (custom_callbacks.py:441-468) on the device: after every env step, the outcomes of the
    envs it reset enter a window of `window_size`; when the window's success rate exceeds capture_radius_sr the
    capture radius of every env shrinks by capture_radius_decay and the window is cleared.  Flavor A.

    `eval_env` (+ eval_freq / n_eval_episodes) gives it the EvalCallback part of the reference's class, whose eval env
    also receives every new radius (:462).  `step_fn(trainer, dev_state, reset_all)` performs one update (default:
    the HIP kernel; CPU tests of the data-parallel protocol pass a host restatement)."""

    def __init__(self, capture_radius_sr, capture_radius_decay, initial_capture_radius, window_size=40,
                 save_path=None, verbose=1, eval_env=None, eval_freq=1000, n_eval_episodes=10, step_fn=None):
        self.sr, self.decay, self.r0 = float(capture_radius_sr), float(capture_radius_decay), float(initial_capture_radius)
        self.window = int(window_size)
        self.save_path, self.verbose = save_path, verbose
        self.step_fn = step_fn or hip_curriculum_step
        self.dev_state = None          # device bytes of a qs_curriculum
        self.host = None               # the last host copy (QsCurriculum)
        self._seen = 0                 # radius reductions already reported
        self._gbuf = None              # the gathered reset_info rows (data parallel)
        self.records = {}              # the logger values the reference records (curriculum/*)
        self.saved = []                # checkpoint paths written
        self.eval_env = eval_env
        self.eval_freq, self.n_eval_episodes = int(eval_freq), int(n_eval_episodes)
        self.evaluator = None
        if eval_env is not None and eval_freq > 0:
            # CurriculumCallback(..., eval_env=eval_env, eval_freq=1000, n_eval_episodes=10) without save paths
            self.evaluator = self._make_evaluator(eval_env, self.eval_freq, self.n_eval_episodes)

    def _make_evaluator(self, eval_env, eval_freq, n_eval_episodes):
        return EvalCallback(eval_env, n_eval_episodes=n_eval_episodes, eval_freq=eval_freq, verbose=self.verbose)

    def _agree_on_evaluator(self, trainer):
        """Data parallel: evaluation is collective (rank 0 evaluates, every rank joins the broadcast of its mean
        reward and a new best's save), so every rank needs an evaluator exactly when rank 0 has one.  EvalCallback
        lets ranks other than 0 pass eval_env=None; here they may also omit it altogether: they get rank 0's
        eval_freq / n_eval_episodes with no env.  A rank with an evaluator when rank 0 has none is refused on every
        rank (all ranks reach the same decision from one all_gather)."""
        if not getattr(trainer, "distributed", False):
            return
        dist = _dist()
        mine = torch.tensor([self.evaluator is not None, self.eval_freq, self.n_eval_episodes], dtype=torch.int64)
        cdev = trainer.device if dist.get_backend(trainer.group) == "nccl" else torch.device("cpu")
        allv = torch.empty(trainer.world_size * 3, dtype=torch.int64, device=cdev)
        dist.all_gather_into_tensor(allv, mine.to(cdev), group=trainer.group)
        allv = allv.cpu().view(trainer.world_size, 3)
        has0, freq0, n0 = (int(v) for v in allv[0])
        if not has0:
            if bool(allv[:, 0].any()):
                raise NAT.QuadSwarmError("DeviceCurriculum: ranks other than 0 have an eval env but rank 0 has "
                                         "none (rank 0 evaluates)")
            return
        if self.evaluator is None:
            self.evaluator = self._make_evaluator(None, freq0, n0)
        elif (self.evaluator.eval_freq, self.evaluator.n_eval_episodes) != (freq0, n0):
            raise NAT.QuadSwarmError("DeviceCurriculum: eval_freq / n_eval_episodes differ from rank 0's")

    @classmethod
    def from_reference_cfg(cls, cfg, save_path=None, **kw):
        """From the reference's QuadrotorEnvConfig (swarm_rl/global_cfg.py: capture_radius_sr, capture_radius_decay,
        initial_capture_radius), as sb_train constructs it (sb_train.py:86-93)."""
        return cls(cfg.capture_radius_sr, cfg.capture_radius_decay, cfg.initial_capture_radius,
                   save_path=save_path, **kw)

    def _init_device(self, trainer, host=None):
        c = host
        if c is None:
            c = NAT.QsCurriculum()
            NAT.check(NAT.lib().qs_curriculum_init(ctypes.byref(c), self.r0, self.sr, self.decay, self.window),
                      "qs_curriculum_init")
        raw = torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8)
        self.dev_state = raw.to(trainer.device)
        self.host = NAT.QsCurriculum.from_buffer_copy(bytes(c))

    def on_training_start(self, trainer):
        if getattr(trainer.env, "cfg", None) is None or trainer.env.cfg.flavor != "A":
            raise NAT.QuadSwarmError("DeviceCurriculum needs a flavor-A env (capture radius)")
        pending = getattr(self, "_pending", None)
        if pending is not None:          # resumed from a trainer checkpoint (the env's radius is in its snapshot)
            self._init_device(trainer, NAT.QsCurriculum.from_buffer_copy(bytes(pending["qs_curriculum"].tolist())))
            self._seen = int(pending["seen"])
            self._pending = None
        elif self.dev_state is None:
            self._init_device(trainer)
            trainer.env.set_capture_radius(self.r0)
            if self.eval_env is not None:
                self.eval_env.set_capture_radius(self.r0)
        self._agree_on_evaluator(trainer)
        if self.evaluator is not None:
            if getattr(self, "_pending_eval", None) is not None:
                self.evaluator.load_state_dict(self._pending_eval)
                self._pending_eval = None
            self.evaluator.on_training_start(trainer)

    def on_step(self, ctx):
        go = True
        if self.evaluator is not None:   # CurriculumCallback._on_step: super()._on_step() first (:443)
            go = self.evaluator.on_step(ctx) is not False
        tr = ctx.trainer
        ri = getattr(tr.env, "reset_info", None)
        if getattr(tr, "distributed", False):
            self._gbuf = gather_env_rows(tr, ri, self._gbuf)
            self.step_fn(tr, self.dev_state, self._gbuf)
        else:
            self.step_fn(tr, self.dev_state, None)
        return go

    def prepare_eval(self, trainer, eval_env):
        # the reference pushes every new radius to its eval env (custom_callbacks.py:462); the eval env only steps
        # inside evaluations, so giving it the current radius right before each one is the same
        if eval_env is self.eval_env and self.dev_state is not None:
            eval_env.set_capture_radius(self.capture_radius)

    def read(self):
        """Host copy of the device state (synchronises)."""
        self.host = NAT.QsCurriculum.from_buffer_copy(bytes(self.dev_state.cpu().numpy().tobytes()))
        return self.host

    @property
    def capture_radius(self):
        return self.read().radius

    def _report(self, trainer):
        c = self.read()
        self.records = {"curriculum/capture_radius": c.radius, "curriculum/sucess_rate": c.success_rate}
        for k in range(self._seen, c.n_shrinks):
            r = c.history[k % NAT.CUR_MAX_HIST]
            if self.verbose and _is_main(trainer):
                print(f"capture radius reduced to:{r}")
            if self.save_path is not None:
                # the reference's name: save_path/curriculum_checkpoint/<radius 0.000 with '_'>.zip; every rank
                # holds the same state, so every rank joins the (collective) save
                p = os.path.join(self.save_path, "curriculum_checkpoint", f"{r:0.3f}".replace(".", "_") + ".pt")
                trainer.save(p)
                self.saved.append(p)
        self._seen = c.n_shrinks

    def on_rollout_end(self, trainer):
        self._report(trainer)

    def on_iteration_end(self, trainer):
        if self.evaluator is not None:
            self.evaluator.on_iteration_end(trainer)

    def on_training_end(self, trainer):
        # reductions of a rollout that a callback stopped (no on_rollout_end) are still logged and checkpointed
        if self.dev_state is not None:
            self._report(trainer)
        if self.evaluator is not None:
            self.evaluator.on_training_end(trainer)

    def state_dict(self):
        sd = {"qs_curriculum": torch.frombuffer(bytearray(bytes(self.read())), dtype=torch.uint8).clone(),
              "seen": self._seen}
        if self.evaluator is not None:
            sd["eval"] = self.evaluator.state_dict()
        return sd

    def load_state_dict(self, sd):
        """Takes effect at the next on_training_start (learn())."""
        self._pending = sd
        self.dev_state = None
        self._pending_eval = sd.get("eval")
        if self.evaluator is not None and self._pending_eval is not None:
            self.evaluator.load_state_dict(self._pending_eval)
            self._pending_eval = None


class CheckpointCallback(TrainerCallback):
    """CheckpointCallback (custom_callbacks.py:131-208): every save_freq env steps a checkpoint named
    {name_prefix}_{num_timesteps}_steps under save_path, as a resumable PPOTrainer checkpoint written at the end of
    the iteration (sb_train uses save_freq = cfg.checkpoint_freq // cfg.num_envs, name_prefix "quad_swarm").
    Every rank counts the same env steps, so every rank joins the same (collective) saves."""

    def __init__(self, save_freq, save_path, name_prefix="rl_model", verbose=0):
        self.save_freq, self.save_path, self.name_prefix, self.verbose = int(save_freq), save_path, name_prefix, verbose
        self.n_calls = 0
        self._due = False
        self.saved = []

    def on_training_start(self, trainer):
        if _is_main(trainer):
            os.makedirs(self.save_path, exist_ok=True)

    def on_step(self, ctx):
        self.n_calls += 1
        if self.n_calls % self.save_freq == 0:
            self._due = True
        return True

    def on_iteration_end(self, trainer):
        if self._due:
            p = os.path.join(self.save_path, f"{self.name_prefix}_{trainer.num_timesteps}_steps.pt")
            trainer.save(p)
            self.saved.append(p)
            if self.verbose >= 2 and _is_main(trainer):
                print(f"Saving model checkpoint to {p}")
            self._due = False

    def state_dict(self):
        return {"n_calls": self.n_calls}

    def load_state_dict(self, sd):
        self.n_calls = int(sd["n_calls"])


def evaluate_policy(policy, env, n_eval_episodes=5, deterministic=True, callback=None):
    """stable_baselines3.common.evaluation.evaluate_policy(model, env, n_eval_episodes, deterministic,
    return_episode_rewards=True) over a device env (SB3 is not installed: restated from its published algorithm,
    parity unpinned against SB3 itself).  The VecEnv's "envs" are the agent rows (SubprocVecEnvCustom: num_envs =
    envs x agents); row i must finish (n_eval_episodes + i) // n_rows episodes; every row steps until all targets
    are met; an episode counts for its row while the row is below its target; rewards accumulate per row in float64.
    callback(i, done, success) is called for every row below its target after every step (SB3's callback(locals,
    globals)); success = the env's reset outcome when the row's episode ended (reset_info), else None.

    Returns (episode_rewards, episode_lengths, episode_successes) in SB3's order (step, then row)."""
    n = env.I
    targets = np.array([(n_eval_episodes + i) // n for i in range(n)], dtype=np.int64)
    counts = np.zeros(n, dtype=np.int64)
    cur_r = np.zeros(n, dtype=np.float64)
    cur_l = np.zeros(n, dtype=np.int64)
    rewards, lengths, successes = [], [], []
    obs = env.reset()
    agents = getattr(env, "N", 1)
    was_training = policy.training
    policy.train(False)
    try:
        while (counts < targets).any():
            with torch.no_grad():
                actions = policy.predict(obs, deterministic=deterministic)
            obs, rew, done, _ = env.step(actions.contiguous())
            r = rew.double().cpu().numpy()
            d = done.cpu().numpy().astype(bool)
            ri = env.reset_info.cpu().numpy() if hasattr(env, "reset_info") else None
            cur_r += r
            cur_l += 1
            for i in range(n):
                if counts[i] < targets[i]:
                    succ = None
                    if d[i] and ri is not None and ri[i // agents] != 0:
                        succ = bool(ri[i // agents] == 2)
                    if callback is not None:
                        callback(i, bool(d[i]), succ)
                    if d[i]:
                        rewards.append(float(cur_r[i]))
                        lengths.append(int(cur_l[i]))
                        successes.append(succ)
                        counts[i] += 1
                        cur_r[i] = 0.0
                        cur_l[i] = 0
    finally:
        policy.train(was_training)
    return rewards, lengths, successes


class EvalCallback(TrainerCallback):
    """EvalCallback (custom_callbacks.py:228-427) for PPOTrainer.learn: every eval_freq env steps, n_eval_episodes
    deterministic episodes on eval_env (evaluate_policy above), `evaluations.npz` under log_path (timesteps, results,
    ep_lengths), the eval/* records, and on a new best mean reward a PPOTrainer checkpoint
    `best_model_save_path/best_model.pt` plus callback_on_new_best.on_new_best(self) (False stops training).
    sb_train: EvalCallback(eval_env, best_model_save_path=logdir/best_model, log_path=logdir/eval,
    eval_freq=cfg.eval_freq // cfg.num_envs, n_eval_episodes=cfg.eval_episodes, deterministic=True) (sb_train.py:76-84).

    eval_env: a device env (QuadSwarmEnv; the reference's eval env is one env of N agents).  Data parallel: only rank 0
    needs one (pass None elsewhere); rank 0's mean reward is broadcast.

    The best model is saved at the end of the iteration in which the new best was found (or at the end of training,
    if learn() stopped first), not mid-rollout: PPOTrainer.save checkpoints are resumable only at the iteration
    boundary (a mid-rollout save would hold num_timesteps / env_steps of a partial rollout without its storage).  The
    weights are the same either way -- the policy changes only in the update."""

    def __init__(self, eval_env, n_eval_episodes=5, eval_freq=10000, log_path=None, best_model_save_path=None,
                 deterministic=True, verbose=1, callback_on_new_best=None):
        self.eval_env = eval_env
        self.n_eval_episodes, self.eval_freq = int(n_eval_episodes), int(eval_freq)
        self.deterministic, self.verbose = deterministic, verbose
        self.best_model_save_path = best_model_save_path
        self.log_path = os.path.join(log_path, "evaluations") if log_path is not None else None
        self.callback_on_new_best = callback_on_new_best
        self.best_mean_reward = -np.inf
        self.last_mean_reward = -np.inf
        self.n_calls = 0
        self.evaluations_results, self.evaluations_timesteps, self.evaluations_length = [], [], []
        self.last_episodes = None      # (rewards, lengths, successes) of the last evaluation (rank 0)
        self.records = {}
        self.best_saved = []
        self._best_due = False

    def on_training_start(self, trainer):
        if _is_main(trainer):
            if self.best_model_save_path is not None:
                os.makedirs(self.best_model_save_path, exist_ok=True)
            if self.log_path is not None:
                os.makedirs(os.path.dirname(self.log_path), exist_ok=True)
            if self.eval_env is None:
                raise NAT.QuadSwarmError("EvalCallback: rank 0 needs an eval env")

    def on_step(self, ctx):
        self.n_calls += 1
        if self.eval_freq > 0 and self.n_calls % self.eval_freq == 0:
            return self.evaluate(ctx.trainer)
        return True

    def evaluate(self, trainer):
        """One evaluation (EvalCallback._on_step's body, :336-418); returns continue_training."""
        main = _is_main(trainer)
        mean = 0.0
        if main:
            for cb in getattr(trainer, "callbacks", ()):
                cb.prepare_eval(trainer, self.eval_env)
            rews, lens, succ = evaluate_policy(trainer.policy, self.eval_env, self.n_eval_episodes, self.deterministic)
            self.last_episodes = (rews, lens, succ)
            if self.log_path is not None:
                self.evaluations_timesteps.append(trainer.num_timesteps)
                self.evaluations_results.append(rews)
                self.evaluations_length.append(lens)
                np.savez(self.log_path, timesteps=self.evaluations_timesteps, results=self.evaluations_results,
                         ep_lengths=self.evaluations_length)
            mean, std = float(np.mean(rews)), float(np.std(rews))
            mlen, slen = float(np.mean(lens)), float(np.std(lens))
            if self.verbose >= 1:
                print(f"Eval num_timesteps={trainer.num_timesteps}, episode_reward={mean:.2f} +/- {std:.2f}")
                print(f"Episode length: {mlen:.2f} +/- {slen:.2f}")
            self.records = {"eval/mean_reward": mean, "eval/mean_ep_length": mlen,
                            "time/total_timesteps": trainer.num_timesteps}
            known = [s for s in succ if s is not None]
            if known:
                self.records["eval/capture_success_rate"] = float(np.mean(known))
        if getattr(trainer, "distributed", False):   # every rank takes rank 0's decision
            t = torch.tensor([mean], dtype=torch.float64, device=trainer.device)
            _dist().broadcast(t, 0, group=trainer.group)
            mean = float(t[0])
        self.last_mean_reward = mean
        go = True
        if mean > self.best_mean_reward:
            if self.verbose >= 1 and main:
                print("New best mean reward!")
            if self.best_model_save_path is not None:
                self._best_due = True          # written at the iteration boundary (on_iteration_end)
            self.best_mean_reward = mean
            if self.callback_on_new_best is not None:
                go = self.callback_on_new_best.on_new_best(self) is not False
        return go

    def _save_best(self, trainer):
        if self._best_due:
            self._best_due = False
            p = os.path.join(self.best_model_save_path, "best_model.pt")
            trainer.save(p)
            self.best_saved.append(p)

    def on_iteration_end(self, trainer):
        self._save_best(trainer)

    def on_training_end(self, trainer):
        self._save_best(trainer)

    def state_dict(self):
        return {"n_calls": self.n_calls, "best_mean_reward": float(self.best_mean_reward),
                "last_mean_reward": float(self.last_mean_reward)}

    def load_state_dict(self, sd):
        self.n_calls = int(sd["n_calls"])
        self.best_mean_reward = float(sd["best_mean_reward"])
        self.last_mean_reward = float(sd["last_mean_reward"])


class StopTrainingOnRewardThreshold:
    """StopTrainingOnRewardThreshold (custom_callbacks.py:496-528) as EvalCallback's callback_on_new_best: stop once
    the best mean reward reaches reward_threshold."""

    def __init__(self, reward_threshold, verbose=0):
        self.reward_threshold, self.verbose = float(reward_threshold), verbose

    def on_new_best(self, eval_cb):
        go = bool(eval_cb.best_mean_reward < self.reward_threshold)
        if self.verbose >= 1 and not go:
            print(f"Stopping training because the mean reward {eval_cb.best_mean_reward:.2f} "
                  f" is above the threshold {self.reward_threshold}")
        return go
