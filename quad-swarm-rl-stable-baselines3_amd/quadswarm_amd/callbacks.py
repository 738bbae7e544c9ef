"""sb_train's training-loop hooks on the device-resident trainer (PPOTrainer.learn).

The reference passes SB3 callbacks to `model.learn` (swarm_rl/sb_train.py:66-103): CheckpointCallback
(swarm_rl/custom_callbacks.py:131-208), EvalCallback, CurriculumCallback (:441-468) and a TensorBoard note.
SB3 calls `callback.on_step()` after every VecEnv step of a rollout, with `training_env.reset_infos` and
`training_env.batch` readable.  Here:

  TrainerCallback   the hook points (on_training_start / on_rollout_start / on_step(ctx) / on_rollout_end /
                    on_iteration_end / on_training_end); on_step returning False stops learn(), like SB3
  StepContext       what on_step sees: the step's device tensors (obs, rewards, dones, actions, reset_info) and,
                    lazily, the reference's host-side `reset_infos` tuple / `batch` (reading reset_infos copies
                    reset_info to the host -- one sync; the device callbacks below never do)
  DeviceCurriculum  CurriculumCallback with its window and radius in device memory: one qs_curriculum_step launch
                    per env step (csrc/qs_curriculum.h), the struct read once per rollout to log and to write the
                    reference's curriculum checkpoints
  CheckpointCallback  the reference's periodic checkpoint (every save_freq env steps, named
                    {name_prefix}_{num_timesteps}_steps), written at the end of the iteration in which the period
                    elapsed as a resumable PPOTrainer checkpoint (PPOTrainer.save)

Differences from the SB3 callbacks (documented, deliberate):
  * checkpoints are written at the rollout / iteration boundary in which the reference would have written them
    mid-rollout.  The policy only changes in the update, so a model saved mid-rollout and at the end of that
    rollout holds the same weights; the iteration boundary is where a trainer checkpoint is resumable.
  * DeviceCurriculum has no eval env to update (the device trainer has no EvalCallback); its radius reaches
    every training env on the device, in the same step as the reference's env_method call.
"""
import ctypes
import os

import torch

from . import _native as NAT


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

    # trainer checkpoints carry every callback's state (PPOTrainer.save / load)
    def state_dict(self):
        return {}

    def load_state_dict(self, sd):
        pass


class StepContext:
    """One env step of a rollout, as on_step sees it (SB3: self.locals + self.training_env).  Device tensors are the
    step's buffers (overwritten by the next step)."""

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


class DeviceCurriculum(TrainerCallback):
    """CurriculumCallback (custom_callbacks.py:441-468) on the device: after every env step, the outcomes of the
    envs it reset enter a window of `window_size`; when the window's success rate exceeds capture_radius_sr the
    capture radius of every env shrinks by capture_radius_decay and the window is cleared.  Flavor A."""

    def __init__(self, capture_radius_sr, capture_radius_decay, initial_capture_radius, window_size=40,
                 save_path=None, verbose=1):
        self.sr, self.decay, self.r0 = float(capture_radius_sr), float(capture_radius_decay), float(initial_capture_radius)
        self.window = int(window_size)
        self.save_path, self.verbose = save_path, verbose
        self.dev_state = None          # device bytes of a qs_curriculum
        self.host = None               # the last host copy (QsCurriculum)
        self._seen = 0                 # radius reductions already reported
        self.records = {}              # the logger values the reference records (curriculum/*)
        self.saved = []                # checkpoint paths written

    @classmethod
    def from_reference_cfg(cls, cfg, save_path=None, **kw):
        """From the reference's QuadrotorEnvConfig (swarm_rl/global_cfg.py: capture_radius_sr, capture_radius_decay,
        initial_capture_radius), as sb_train constructs it (sb_train.py:82-89)."""
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

    def on_step(self, ctx):
        env = ctx.trainer.env
        st = ctypes.c_void_p(torch.cuda.current_stream(ctx.trainer.device).cuda_stream)
        NAT.check(NAT.lib().qs_curriculum_step(env._h, ctypes.c_void_p(self.dev_state.data_ptr()), st),
                  "qs_curriculum_step")
        return True

    def read(self):
        """Host copy of the device state (synchronises)."""
        self.host = NAT.QsCurriculum.from_buffer_copy(bytes(self.dev_state.cpu().numpy().tobytes()))
        return self.host

    @property
    def capture_radius(self):
        return self.read().radius

    def on_rollout_end(self, trainer):
        c = self.read()
        self.records = {"curriculum/capture_radius": c.radius, "curriculum/sucess_rate": c.success_rate}
        for k in range(self._seen, c.n_shrinks):
            r = c.history[k % NAT.CUR_MAX_HIST]
            if self.verbose:
                print(f"capture radius reduced to:{r}")
            if self.save_path is not None:
                # the reference's name: save_path/curriculum_checkpoint/<radius 0.000 with '_'>.zip
                p = os.path.join(self.save_path, "curriculum_checkpoint", f"{r:0.3f}".replace(".", "_") + ".pt")
                trainer.save(p)
                self.saved.append(p)
        self._seen = c.n_shrinks

    def state_dict(self):
        return {"qs_curriculum": torch.frombuffer(bytearray(bytes(self.read())), dtype=torch.uint8).clone(),
                "seen": self._seen}

    def load_state_dict(self, sd):
        """Takes effect at the next on_training_start (learn())."""
        self._pending = sd
        self.dev_state = None


class CheckpointCallback(TrainerCallback):
    """CheckpointCallback (custom_callbacks.py:131-208): every save_freq env steps a checkpoint named
    {name_prefix}_{num_timesteps}_steps under save_path, as a resumable PPOTrainer checkpoint written at the end of
    the iteration (sb_train uses save_freq = cfg.checkpoint_freq // cfg.num_envs, name_prefix "quad_swarm")."""

    def __init__(self, save_freq, save_path, name_prefix="rl_model", verbose=0):
        self.save_freq, self.save_path, self.name_prefix, self.verbose = int(save_freq), save_path, name_prefix, verbose
        self.n_calls = 0
        self._due = False
        self.saved = []

    def on_training_start(self, trainer):
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
            if self.verbose >= 2:
                print(f"Saving model checkpoint to {p}")
            self._due = False

    def state_dict(self):
        return {"n_calls": self.n_calls}

    def load_state_dict(self, sd):
        self.n_calls = int(sd["n_calls"])
