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
  * native (as_torch=True): torch device tensors in/out, nothing crosses PCIe.  Its infos are lazy (a
    contract change, see StepInfos): read them before the next step_wait.
"""
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


class StepInfos(Sequence):
    """infos of one step, len == num_envs (agent rows).  Rows of finished envs get terminal_observation (and
    episode_extra_stats, quadrotor_multi.py:739-831, when the env keeps them).  With per-step infos on, every row
    carries the reference's per-agent entries: flavor B {"rewards": {...}} (quadrotor_single.py:79-105, 371;
    quadrotor_multi.py:642-651), flavor A {"rewards": {}, "goal_dist": ...} (quadrotor_single_rewards.py:457);
    their dicts are built when a row is read, so a 32k-agent step does not build 32k dicts.  A row's dict is built
    once and kept: infos[i] returns the same mutable dict every time, so in-place writes (SB3's VecNormalize
    rewriting terminal_observation, a wrapper adding episode_extra_stats) stick, as with the reference's list.

    Native mode builds it lazily -- a contract change against the reference's eager list: nothing is copied to the
    host until a row (or the done rows) is read, and that first read must happen before the next step_wait (the
    device buffers it reads are the step's; a later first read raises RuntimeError).  Rows read in time stay
    valid: their terminal_observation is a copy of the finished agents' rows, not a view of the env's buffer."""

    def __init__(self, n, done_rows=(), term=None, extra=None, rewards=None, goal_dist=None, resolve=None):
        self._n = n
        self._resolve = resolve
        self._d = None
        self._m = {}       # row -> the dict handed out for it (memoised)
        if resolve is None:
            self._build(done_rows, term, extra, rewards, goal_dist)

    def _build(self, done_rows, term, extra, rewards, goal_dist):
        """term: the terminal observations of the finished rows, in done_rows order."""
        self._rows = np.asarray(done_rows, dtype=np.int64)
        self._rewards, self._gd = rewards, goal_dist
        self._d = {}
        for k, r in enumerate(self._rows.tolist()):
            self._d[r] = {"terminal_observation": term[k], "TimeLimit.truncated": False}
            if extra is not None:
                self._d[r]["episode_extra_stats"] = extra[k]

    def _ready(self):
        if self._d is None:
            self._build(*self._resolve())
            self._resolve = None

    @property
    def done_rows(self):
        """Agent rows of the envs that finished in this step (host int64 array)."""
        self._ready()
        return self._rows

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        row = self._m.get(i)
        if row is not None:
            return row
        self._ready()
        row = self._d.get(i)
        if row is None:
            row = {}
        if self._rewards is not None:
            from .infos import rewards_dict
            row["rewards"] = rewards_dict(self._rewards, i)
        elif self._gd is not None:
            row["rewards"] = {}
            row["goal_dist"] = float(self._gd[i])
        self._m[i] = row
        return row


class GpuQuadVecEnv:
    """raise_on_nan: like QuadrotorSingle's reward check (quadrotor_single.py:87-90), raise ValueError when a
    step produced a non-finite reward (the kernels' qs_counters guard).  Compat mode checks every step when it
    reads the step's results; native mode never waits for the device: it polls a stream-ordered copy of the
    counter and raises at the first step_wait that finds it increased (at most a few steps late).
    infos: per-step infos (config step_infos): infos[i]["rewards"] (flavor B) / infos[i]["goal_dist"] (flavor A)
    on every agent row, like the reference's step."""

    def __init__(self, cfg: QuadSwarmConfig = None, as_torch=False, device=None, raise_on_nan=True, infos=True,
                 **cfg_over):
        cfg = cfg or QuadSwarmConfig()
        for k, v in cfg_over.items():
            setattr(cfg, k, v)
        if infos:
            cfg.step_infos = True
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
        self._reset_infos = tuple(None for _ in range(cfg.num_envs))
        self._last_infos = None
        self._actions = None
        self.render_mode = None
        self.raise_on_nan = raise_on_nan
        self._nan_last = 0      # the non-finite reward counter as last read
        self._gen = 0           # step counter: lazy infos of an older step refuse to resolve
        self._nan_host = self._nan_ev = None
        if as_torch:            # a pinned slot + event for the stream-ordered counter copy (native mode)
            import torch
            self._nan_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._nan_ev = torch.cuda.Event()
            self._nan_pending = False

    # ---- VecEnv API ----
    def reset(self):
        obs = self.env.reset()
        if self.cfg.flavor == "A":
            ri = self.env.reset_info.cpu().numpy()
            self._reset_infos = tuple({"success": bool(v == 2)} for v in ri)
        else:
            self._reset_infos = tuple({} for _ in range(self.cfg.num_envs))
        self._last_infos = None
        return obs if self.as_torch else obs.cpu().numpy()

    @property
    def reset_infos(self):
        """Per env: {"success": bool} (flavor A) / {} (flavor B) when the env was reset by the last call, else None
        (SubprocVecEnvCustom.reset_infos, subproc_vec_env_custom.py:152, 162).  Native mode computes it on first
        read after a step."""
        if self._last_infos is not None:
            self._reset_infos = self._reset_infos_of(self._last_infos.done_rows)
            self._last_infos = None
        return self._reset_infos

    @reset_infos.setter
    def reset_infos(self, v):
        self._reset_infos, self._last_infos = v, None

    def step_async(self, actions):
        self._actions = actions
        self.waiting = True

    def _check_nan(self, value):
        """Raise on any increase of the non-finite reward counter since the last read; a drop means it was
        reset (qs_counters_reset through any path): resynchronise."""
        v = int(value)
        last, self._nan_last = self._nan_last, v
        if self.raise_on_nan and v > last:
            raise ValueError("QuadEnv: reward is Nan")

    def step_wait(self):
        import torch

        if self.as_torch and self._nan_pending and self._nan_ev.query():   # the previous copy has landed
            self._nan_pending = False
            self._check_nan(self._nan_host[0])
        obs, rew, done, term = self.env.step(self._actions)
        self.waiting = False
        self.batch += 1
        self._gen += 1
        d = done.bool()
        if self.as_torch:
            # nothing leaves the device here: the counter is copied stream-ordered into pinned memory, the
            # infos resolve on first read
            if not self._nan_pending:
                self._nan_host.copy_(self.env.stats[N.ST_REW:N.ST_REW + 1], non_blocking=True)
                self._nan_ev.record()
                self._nan_pending = True
            gen = self._gen
            comp = self.env.rew_info.clone() if self.env.rew_info is not None else None

            def resolve():
                if gen != self._gen:
                    raise RuntimeError("GpuQuadVecEnv infos of an older step: read them before the next step_wait")
                rows_t = torch.nonzero(d).flatten()
                rows = rows_t.cpu().numpy()
                return (rows, term[rows_t].clone(), self._episode_extra_stats(rows) if len(rows) else None) + \
                    self._step_info_columns(comp)
            infos = StepInfos(self.num_envs, resolve=resolve)
            self._last_infos = infos
            return obs, rew, d, infos
        # compat: one small D2H read (like the pipes' recv): the finished rows and the non-finite reward counter
        h = torch.cat([torch.nonzero(d).flatten(), self.env.stats[N.ST_REW:N.ST_REW + 1]]).cpu().numpy()
        rows = h[:-1]
        self._check_nan(h[-1])
        self._reset_infos, self._last_infos = self._reset_infos_of(rows), None
        extra = self._episode_extra_stats(rows) if len(rows) else None
        term_np = term[torch.as_tensor(rows, device=term.device)].cpu().numpy() if len(rows) else None
        cols = self._step_info_columns(self.env.rew_info)
        return obs.cpu().numpy(), rew.cpu().numpy(), d.cpu().numpy(), StepInfos(self.num_envs, rows, term_np, extra,
                                                                               *cols)

    def _step_info_columns(self, comp):
        """(flavor-B reward columns, flavor-A goal distances) of a step's reward components (None when off)."""
        if comp is None:
            return None, None
        c = comp.cpu().numpy()
        if self.cfg.flavor == "A":
            return None, c[N.RI_GOAL_DIST]
        from .infos import reward_columns_b
        return reward_columns_b(c, self.env.reward_coefficients(), float(self.cfg.dt), self.cfg.use_obstacles), None

    def _episode_extra_stats(self, rows):
        """infos[i]["episode_extra_stats"] of the finished rows: the env's counters (quadrotor_multi.py:739-831)
        and, with experience replay on, the wrapper's "replay/*" values (quad_experience_replay.py:124-137)."""
        from .stats import episode_extra_stats
        out = [{} for _ in rows]
        if self.env.estats is not None:
            est = self.env.estats[self.env._torch.as_tensor(rows, device=self.env.device, dtype=self.env._torch.long)].cpu().numpy()
            for k in range(len(rows)):
                out[k] = episode_extra_stats(est[k], use_obstacles=self.cfg.use_obstacles)
        if self.env.replay is not None:
            rs = self.env.replay_stats()
            envs = np.asarray(rows) // self.agents_per_env
            nrep = self.env.replay["nrep"].cpu().numpy()
            perm = self.env.replay["perm"].cpu().numpy()
            es = self.env.env_state.cpu().numpy()
            c = self.cfg
            dens, sizes = [c.obst_density], [c.obst_size]     # table index 0 = the configured values
            if c.use_obstacles and c.domain_random_active:
                d, _, z = c.domain_random_tables()
                dens, sizes = dens + [float(x) for x in d], sizes + [float(x) for x in z]
            ri = self.env.replay["ri"].cpu().numpy()
            for k, e in enumerate(envs):
                n = int(rs["replay/replay_buffer_size"][e])
                if c.use_obstacles:      # the density / size the env's new episode runs with (:113-116, :186-211)
                    od, osz = dens[int(es[N.E_OBST_M, e])], sizes[int(es[N.E_OBST_SZ, e])]
                else:                    # curr_obst_density drops to 0.0 at the env's first replay (:187-190)
                    od, osz = (0.0 if ri[N.R_REPLAYED, e] > 0 else c.obst_density), c.obst_size
                out[k].update({"replay/replay_rate": float(rs["replay/replay_rate"][e]),
                               "replay/new_episode_rate": float(rs["replay/new_episode_rate"][e]),
                               "replay/replay_buffer_size": n,
                               "replay/avg_replayed": float(np.mean(nrep[perm[:n, e], e])) if n else 0,
                               "replay/obst_density": od, "replay/obst_size": osz})
        return out

    def counters(self):
        """The step kernels' non-finite guard counters (qs_counters) since creation or reset_counters()."""
        return self.env.counters()

    def reset_counters(self):
        if self.as_torch and self._nan_pending:   # a copy still in flight carries the count from before the reset
            self._nan_ev.synchronize()
            self._nan_pending = False
        self.env.reset_counters()
        self._nan_last = 0

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _reset_infos_of(self, done_rows):
        if len(done_rows) == 0:
            return (None,) * self.cfg.num_envs
        envs = sorted(set(int(r) // self.agents_per_env for r in np.asarray(done_rows).tolist()))
        ri = [None] * self.cfg.num_envs
        if self.cfg.flavor == "A":
            flags = self.env.reset_info.cpu().numpy()
            for e in envs:
                ri[e] = {"success": bool(flags[e] == 2)}
        else:
            for e in envs:
                ri[e] = {}
        return tuple(ri)

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
