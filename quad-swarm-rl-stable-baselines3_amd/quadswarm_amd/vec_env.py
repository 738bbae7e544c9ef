"""GpuQuadVecEnv: the SubprocVecEnvCustom surface over the HBM-resident swarm step.

Mirrors swarm_rl/env_wrappers/subproc_vec_env_custom.py:88-248 so that sb_train's
`SubprocVecEnvCustom([make_env]*num_envs, agents_per_env=N)` (swarm_rl/sb_train.py:50-51) can be
swapped for `GpuQuadVecEnv(cfg)`:
  num_envs = envs * agents_per_env                        (:139)
  step_async(actions (num_envs, act_dim))                 (:141-147)
  step_wait() -> obs, rews, dones, infos                  (:149-153)
  infos[i]["terminal_observation"] for every agent of a finished env, which is reset (:42-46)
  reset_infos: per env, after a reset {} (flavor B) or {"success": bool} (flavor A,
               quadrotor_multi_rewards.py:625-627), else None (:152, :162)
  env_method("set_capture_radius", r, indices=...)      (custom_callbacks.py:455-462, flavor A)
  env_method / get_attr / set_attr / has_attr over ENV indices (:212-237)
Two modes:
  * compat (default): numpy in/out, exactly the reference's types (obs float32 instead of float64;
    the policy casts to float32 anyway, ActorCriticPolicyCustom.py:463);
  * native (as_torch=True): torch device tensors in/out, nothing crosses PCIe.
"""
import types
from collections.abc import Sequence

import numpy as np

from . import _native as N
from .config import QuadSwarmConfig
from .env import QuadSwarmEnv, observation_bounds

try:  # the reference's space type when gymnasium is installed
    from gymnasium import spaces as _spaces
except Exception:  # pragma: no cover - exercised where gymnasium is absent
    _spaces = None


class Box:
    """Minimal stand-in for gymnasium.spaces.Box (used only when gymnasium is absent)."""

    def __init__(self, low, high, dtype=np.float32):
        self.low, self.high = np.asarray(low, dtype=dtype), np.asarray(high, dtype=dtype)
        self.shape, self.dtype = self.low.shape, np.dtype(dtype)

    def sample(self):
        return np.random.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


def make_box(low, high):
    if _spaces is not None:
        return _spaces.Box(low, high, dtype=np.float32)
    return Box(low, high)


_EMPTY = types.MappingProxyType({})


class StepInfos(Sequence):
    """infos of one step, len == num_envs (agent rows).  Rows of finished envs get a fresh dict with
    terminal_observation; every other row is a shared read-only empty mapping, so a 32k-agent step
    does not build 32k dicts."""

    def __init__(self, n, done_rows=(), term=None):
        self._n = n
        self._d = {}
        for r in done_rows:
            self._d[int(r)] = {"terminal_observation": term[int(r)], "TimeLimit.truncated": False}

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        return self._d.get(i, _EMPTY)


class GpuQuadVecEnv:
    def __init__(self, cfg: QuadSwarmConfig = None, as_torch=False, device=None, **cfg_over):
        cfg = cfg or QuadSwarmConfig()
        for k, v in cfg_over.items():
            setattr(cfg, k, v)
        self.cfg = cfg
        self.env = QuadSwarmEnv(cfg, device=device)
        self.agents_per_env = cfg.num_agents
        self.num_envs = cfg.num_envs * cfg.num_agents
        lo, hi = observation_bounds(cfg)
        self.observation_space = make_box(lo, hi)
        ad = cfg.act_dim   # CustomPidControl.action_space (quadrotor_control.py:74-86) is (2,) in flavor A
        self.action_space = make_box(-np.ones(ad, np.float32), np.ones(ad, np.float32))
        self.as_torch = as_torch
        self.batch = 0
        self.waiting = False
        self.closed = False
        self.reset_infos = tuple(None for _ in range(cfg.num_envs))
        self._actions = None
        self.render_mode = None

    # ---- VecEnv API ----
    def reset(self):
        obs = self.env.reset()
        if self.cfg.flavor == "A":
            ri = self.env.reset_info.cpu().numpy()
            self.reset_infos = tuple({"success": bool(v == 2)} for v in ri)
        else:
            self.reset_infos = tuple({} for _ in range(self.cfg.num_envs))
        return obs if self.as_torch else obs.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions
        self.waiting = True

    def step_wait(self):
        import torch

        obs, rew, done, term = self.env.step(self._actions)
        self.waiting = False
        self.batch += 1
        d = done.bool()
        rows = torch.nonzero(d).flatten().cpu().numpy()   # one small D2H sync (like the pipes' recv)
        self._set_reset_infos(rows)
        if self.as_torch:
            return obs, rew, d, StepInfos(self.num_envs, rows, term)
        term_np = term.cpu().numpy() if len(rows) else None
        return obs.cpu().numpy(), rew.cpu().numpy(), d.cpu().numpy(), StepInfos(self.num_envs, rows, term_np)

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _set_reset_infos(self, done_rows):
        if len(done_rows) == 0:
            self.reset_infos = (None,) * self.cfg.num_envs
            return
        envs = sorted(set(int(r) // self.agents_per_env for r in np.asarray(done_rows).tolist()))
        ri = [None] * self.cfg.num_envs
        if self.cfg.flavor == "A":
            flags = self.env.reset_info.cpu().numpy()
            for e in envs:
                ri[e] = {"success": bool(flags[e] == 2)}
        else:
            for e in envs:
                ri[e] = {}
        self.reset_infos = tuple(ri)

    def close(self):
        if not self.closed:
            self.env.close()
            self.closed = True

    def seed(self, seed=None):
        if seed is not None:
            self.env.set_param("seed", int(seed))
        return [seed] * self.cfg.num_envs

    # ---- env indices (not agent rows), like SubprocVecEnvCustom._get_indices (:226-237) ----
    def _get_indices(self, indices):
        if indices is None:
            return range(self.cfg.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = list(self._get_indices(indices))
        if method_name in ("set_param", "set_reward_coeff"):
            self.env.set_param(*method_args, **method_kwargs)
            return [None] * len(idx)
        if method_name == "set_capture_radius":
            self.env.set_capture_radius(*method_args, env_indices=None if indices is None else idx)
            return [None] * len(idx)
        raise AttributeError(f"unknown env method {method_name}")

    def get_attr(self, attr_name, indices=None):
        idx = list(self._get_indices(indices))
        if attr_name in ("num_agents", "agents_per_env"):
            return [self.cfg.num_agents] * len(idx)
        if attr_name == "cfg":
            return [self.cfg] * len(idx)
        if attr_name == "capture_radius" and self.cfg.flavor == "A":
            r = self.env.env_f[N.ENVF_CAPTURE].cpu().numpy()
            return [float(r[i]) for i in idx]
        if hasattr(self.cfg, attr_name):
            return [getattr(self.cfg, attr_name)] * len(idx)
        raise AttributeError(attr_name)

    def set_attr(self, attr_name, value, indices=None):
        if attr_name.startswith("rew_") or attr_name in ("quadcol_bin", "quadcol_bin_smooth_max", "quadcol_bin_obst", "ep_len"):
            self.env.set_param(attr_name, value)
            return
        setattr(self.cfg, attr_name, value)

    def has_attr(self, attr_name):
        try:
            self.get_attr(attr_name, indices=[0])
            return True
        except AttributeError:
            return False

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(list(self._get_indices(indices)))


def make_vec_env(cfg=None, **kw):
    """Factory used where sb_train builds SubprocVecEnvCustom (sb_train.py:50-51)."""
    if cfg is not None and not isinstance(cfg, QuadSwarmConfig):
        cfg = QuadSwarmConfig.from_reference_cfg(cfg)
    return GpuQuadVecEnv(cfg, **kw)


__all__ = ["GpuQuadVecEnv", "StepInfos", "make_vec_env", "Box"]
