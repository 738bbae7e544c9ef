"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): host restatement of sb_train's capture-radius
curriculum, CurriculumCallback._on_step (swarm_rl/custom_callbacks.py:441-468), minus its logging and eval env.

`CurriculumOracle.step(resets)` takes one VecEnv step's reset_infos in env order -- None for an env the step did
not reset, else {"success": bool} (or the device code's reset_info byte: 0 none, 1 failure, 2 success) -- exactly as
the reference iterates `self.training_env.reset_infos` (:452-456): every reset env writes its outcome into the
window at window_i % window_size and advances window_i; if any env was reset, sucess_rate = sum(window) /
window_size (:458) and above capture_radius_sr the radius is multiplied by capture_radius_decay (:459-460) and the
window cleared (:464).  fp64 like the reference's numpy / Python floats.

Parity is pinned by the GPU test against the HIP kernel (tests/test_gpu_trainer.py) and, here, by the reference
lines themselves: the callback is a dozen lines of numpy with no library call beyond np.sum / np.zeros."""
import numpy as np


class CurriculumOracle:
    def __init__(self, initial_radius, sr_threshold, decay, window=40):
        self.W = int(window)
        self.past = np.zeros(self.W)          # past_successes (:437)
        self.window_i = 0                     # :436
        self.success_rate = 0.0               # sucess_rate (:438)
        self.radius = float(initial_radius)   # current_capture_radius (:439)
        self.sr, self.decay = float(sr_threshold), float(decay)
        self.history = []                     # radius after each reduction (the curriculum checkpoints' names)

    def step(self, resets):
        change = False
        for e in resets:
            if isinstance(e, (int, np.integer)):
                e = None if e == 0 else {"success": e == 2}
            if e is not None:
                self.past[self.window_i % self.W] = e["success"]
                self.window_i += 1
                change = True
        if change:
            self.success_rate = np.sum(self.past) / self.W
            if self.success_rate > self.sr:
                self.radius = self.decay * self.radius
                self.history.append(self.radius)
                self.past = np.zeros(self.W)
                return True
        return False
