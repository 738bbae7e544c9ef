"""Batched, HBM-resident QuadrotorEnvMulti: E envs x N drones stepped by one HIP launch.

Flavor B follows quadrotor_multi.QuadrotorEnvMulti.step / reset (gym_art/quadrotor_multi/quadrotor_multi.py:
440-841) with its in-env auto-reset (:739-838); flavor A follows quadrotor_multi_rewards.QuadrotorEnvMulti
(quadrotor_multi_rewards.py:541-991) plus the worker-side reset on done.  Both keep the SubprocVecEnvCustom
terminal_observation / reset_infos contract (swarm_rl/env_wrappers/subproc_vec_env_custom.py:33-52).
All buffers are torch tensors viewing one device workspace that libquadswarm.so reads and writes in place
(zero-copy).
"""
import ctypes

import numpy as np

from . import _native as N
from .config import QuadSwarmConfig


class QuadSwarmEnv:
    def __init__(self, cfg: QuadSwarmConfig, device=None):
        import torch

        self.cfg = cfg
        self.device = torch.device(device if device is not None else cfg.device)
        if self.device.type != "cuda" or not torch.cuda.is_available():
            raise N.QuadSwarmError("QuadSwarmEnv needs a HIP device (torch.cuda on ROCm)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.qcfg = cfg.to_qs_config()
        L = N.lib()
        lay = N.QsLayout()
        N.check(L.qs_layout_query(self.qcfg, lay), "qs_layout_query")
        self.layout = lay
        self.E, self.N = cfg.num_envs, cfg.num_agents
        self.I = self.E * self.N
        self.obs_dim = lay.obs_dim
        # qs_create zero-fills and initialises the workspace on the null stream: allocate without a fill
        # kernel and drain the device first, so no pending work of another (non-blocking) stream on
        # recycled caching-allocator memory can land after the initialisation
        self._raw = torch.empty(lay.total_bytes + 256, dtype=torch.uint8, device=self.device)
        off = (-self._raw.data_ptr()) % 256
        ws = self._raw[off:off + lay.total_bytes]
        self._ws = ws
        torch.cuda.synchronize(self.device)
        h = ctypes.c_void_p()
        N.check(L.qs_create(self.qcfg, self.device.index, ctypes.c_void_p(ws.data_ptr()), ctypes.byref(h)), "qs_create")
        self._h = h
        if cfg.specialize:
            try:
                self.specialize(True)
            except N.QuadSwarmError as e:   # the generic HIP kernels give the same results (bitwise)
                import warnings
                warnings.warn(f"qs_specialize failed, using the generic kernels: {e}")

        def view(o, nbytes, dtype, shape):
            return ws[o:o + nbytes].view(dtype).view(*shape)
        E, I, od = self.E, self.I, self.obs_dim
        self.state = view(lay.state, 4 * N.NF * I, torch.float32, (N.NF, I))
        self.istate = view(lay.istate, 4 * N.NI * I, torch.int32, (N.NI, I))
        self.env_state = view(lay.env, 4 * N.NE * E, torch.int32, (N.NE, E))
        self.env_f = view(lay.env_f, 4 * N.NENVF * E, torch.float32, (N.NENVF, E))
        self.reset_info = view(lay.reset_info, E, torch.uint8, (E,))
        M = cfg.max_obstacles if cfg.use_obstacles else 0   # pillar slots (an env uses its first QS_E_OBST_M)
        self.obstacles = view(lay.obst, 8 * M * E, torch.float32, (E, M, 2)) if M else None
        self.stale_vel = view(lay.stale_vel, 4 * 3 * I, torch.float32, (3, I))
        self.obs = view(lay.obs, 4 * I * od, torch.float32, (I, od))
        self.term_obs = view(lay.term_obs, 4 * I * od, torch.float32, (I, od))
        self.rew = view(lay.rew, 4 * I, torch.float32, (I,))
        self.done = view(lay.done, I, torch.uint8, (I,))
        self.stats = view(lay.stats, 8 * N.NSTAT, torch.int64, (N.NSTAT,))
        from .stats import NES
        # episode_extra_stats rows [I, QS_NES] (written for the drones of envs that finished in a step)
        self.estats = view(lay.estats, 4 * NES * I, torch.float32, (I, NES)) if self.qcfg.episode_stats else None
        # the last step's reward components [QS_NRI, I] (config step_infos; quadswarm_amd.infos builds the dicts)
        self.rew_info = view(lay.rew_info, 4 * N.NRI * I, torch.float32, (N.NRI, I)) if self.qcfg.step_infos else None
        self.act_dim = cfg.act_dim
        self._align = 8 if cfg.flavor == "A" else 16
        # the reward coefficients the kernels use, as the host set them (float64: what the reference's rew_coeff
        # holds; infos[i]["rewards"] is built with them)
        r = cfg.rew_coeff
        self._coeff = {"pos": r.get("pos", 1.0), "effort": r.get("effort", 0.05), "crash": r.get("crash", 1.0),
                       "orient": r.get("orient", 1.0), "spin": r.get("spin", 0.1),
                       "quadcol_bin": float(cfg.collision_reward), "quadcol_bin_obst": float(cfg.obst_collision_reward)}
        self._torch = torch
        self.replay = None
        if cfg.replay_buffer_sample_prob > 0:
            self.enable_replay(cfg.replay_buffer_sample_prob)

    # ------------------------------------------------------------------------------------------
    def enable_replay(self, sample_prob=0.75, **over):
        """ExperienceReplayWrapper on device (quad_experience_replay.py:66-216): per-env checkpoints, collision
        events and replayed episodes, run by qs_step / qs_reset from now on.  `over` overrides fields of the
        reference-derived qs_replay_config (cp_every, grace_ticks, min_gap_ticks, buffer_size, ...)."""
        rc = N.QsReplayConfig()
        N.check(N.lib().qs_replay_config_default(ctypes.byref(rc), float(self.qcfg.control_dt)), "qs_replay_config_default")
        rc.sample_prob = float(sample_prob)
        for k, v in over.items():
            setattr(rc, k, v)
        nb = ctypes.c_size_t()
        N.check(N.lib().qs_replay_workspace_bytes(self._h, ctypes.byref(rc), ctypes.byref(nb)), "qs_replay_workspace_bytes")
        raw = self._torch.empty(nb.value + 256, dtype=self._torch.uint8, device=self.device)
        off = (-raw.data_ptr()) % 256
        ws = raw[off:off + nb.value]
        self._torch.cuda.synchronize(self.device)   # qs_replay_enable initialises it synchronously
        N.check(N.lib().qs_replay_enable(self._h, ctypes.byref(rc), ctypes.c_void_p(ws.data_ptr())), "qs_replay_enable")
        rb = N.QsReplayBuffers()
        N.check(N.lib().qs_replay_buffers_get(self._h, ctypes.byref(rb)), "qs_replay_buffers_get")
        self.replay_config, self._replay_ws = rc, ws
        self.replay = _replay_views(self._torch, ws, rb, rc, self.E)

    def disable_replay(self):
        self._torch.cuda.synchronize(self.device)
        N.check(N.lib().qs_replay_disable(self._h), "qs_replay_disable")
        self.replay = None

    def replay_stats(self):
        """The wrapper's episode_extra_stats "replay/*" values (quad_experience_replay.py:133-140), per env."""
        if self.replay is None:
            return None
        ri = self.replay["ri"].cpu().numpy()
        ep = np.maximum(ri[N.R_EPISODES], 1)
        return {"replay/replay_rate": ri[N.R_REPLAYED] / ep,
                "replay/new_episode_rate": (ri[N.R_EPISODES] - ri[N.R_REPLAYED]) / ep,
                "replay/replay_buffer_size": ri[N.R_BUF_N].copy()}

    # ------------------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self._torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, env_mask=None):
        """QuadrotorEnvMulti.reset for all envs (or those with env_mask[e] != 0); returns obs [I, obs_dim]."""
        m = None
        if env_mask is not None:
            m = self._torch.as_tensor(env_mask, device=self.device).to(self._torch.uint8).contiguous()
            if m.numel() != self.E:
                raise ValueError("env_mask must have num_envs entries")
        N.check(N.lib().qs_reset(self._h, ctypes.c_void_p(m.data_ptr()) if m is not None else None, self._stream()),
                "qs_reset")
        self._mask_keepalive = m
        return self.obs

    def step(self, actions):
        """One control step of every env.  actions: [E*N, act_dim] (or [E, N, act_dim]) raw policy output
        (act_dim 4 for flavor B, 2 for flavor A).

        Returns device views (obs, rew, done, term_obs); they are overwritten by the next call.
        reset_info[e] (0 none, 1 {"success": False}, 2 {"success": True}) says which envs were reset."""
        a = actions
        if not (self._torch.is_tensor(a) and a.device == self.device and a.dtype == self._torch.float32
                and a.is_contiguous() and a.data_ptr() % self._align == 0):
            a = self._torch.as_tensor(a, device=self.device, dtype=self._torch.float32).contiguous()
        if a.numel() != self.I * self.act_dim:
            raise ValueError(f"actions must have {self.I * self.act_dim} elements, got {a.numel()}")
        self._act_keepalive = a
        N.check(N.lib().qs_step(self._h, ctypes.c_void_p(a.data_ptr()), self._stream()), "qs_step")
        return self.obs, self.rew, self.done, self.term_obs

    def step_n(self, actions, steps):
        """`steps` back-to-back steps with the same action buffer from one C call (qs_step_n): the
        benchmark's eager launch loop.  actions must already be a contiguous aligned fp32 device tensor."""
        a = actions
        if not (self._torch.is_tensor(a) and a.device == self.device and a.dtype == self._torch.float32
                and a.is_contiguous() and a.data_ptr() % self._align == 0 and a.numel() == self.I * self.act_dim):
            raise ValueError("step_n: actions must be a contiguous, aligned fp32 device tensor of I * act_dim")
        self._act_keepalive = a
        N.check(N.lib().qs_step_n(self._h, ctypes.c_void_p(a.data_ptr()), int(steps), self._stream()), "qs_step_n")
        return self.obs, self.rew, self.done, self.term_obs

    def counters(self):
        """Non-finite guard counters (qs_counters): {"nonfinite_obs", "nonfinite_rew", "nonfinite_state"}
        accumulated by every step since creation / reset_counters().  Synchronises the current stream."""
        st = N.QsStats()
        N.check(N.lib().qs_counters(self._h, ctypes.byref(st), self._stream()), "qs_counters")
        return {"nonfinite_obs": st.nonfinite_obs, "nonfinite_rew": st.nonfinite_rew,
                "nonfinite_state": st.nonfinite_state}

    def reset_counters(self):
        N.check(N.lib().qs_counters_reset(self._h, self._stream()), "qs_counters_reset")

    def specialize(self, enable=True):
        """Switch to kernels recompiled (hipRTC) with this env's parameters as constants (qs_specialize);
        same results as the generic kernels, shorter per-step critical path."""
        N.check(N.lib().qs_specialize(self._h, 1 if enable else 0), "qs_specialize")

    @property
    def specialized(self):
        return bool(N.lib().qs_is_specialized(self._h))

    # ------------------------------------------------------------------------------------------
    _COEFF_PARAMS = {"rew_pos": "pos", "rew_effort": "effort", "rew_crash": "crash", "rew_orient": "orient",
                     "rew_spin": "spin", "quadcol_bin": "quadcol_bin", "quadcol_bin_obst": "quadcol_bin_obst"}

    def set_param(self, key, value):
        N.check(N.lib().qs_set_param(self._h, key.encode(), float(value)), "qs_set_param")
        if key in self._COEFF_PARAMS:
            self._coeff[self._COEFF_PARAMS[key]] = float(value)

    def reward_coefficients(self):
        """The reward coefficients of the next step (rew_coeff + quadcol_bin / quadcol_bin_obst), float64."""
        return dict(self._coeff)

    def get_param(self, key):
        v = ctypes.c_double()
        N.check(N.lib().qs_get_param(self._h, key.encode(), ctypes.byref(v)), "qs_get_param")
        return v.value

    def set_capture_radius(self, value, env_indices=None):
        """QuadrotorEnvMulti.set_capture_radius (quadrotor_multi_rewards.py:212-213) for all envs or a subset;
        the radius lives in device memory, so captured graphs see it."""
        if self.cfg.flavor != "A":
            raise N.QuadSwarmError("set_capture_radius is a flavor-A method")
        if env_indices is None:
            self.set_param("capture_radius", value)
        else:
            idx = self._torch.as_tensor(list(env_indices), dtype=self._torch.long, device=self.device)
            self.env_f[N.ENVF_CAPTURE].index_fill_(0, idx, float(value))

    def get_state(self):
        """Host snapshot (bytes) of the full env state + RNG counter (checkpoint / replay)."""
        n = N.lib().qs_state_bytes(self._h)
        buf = (ctypes.c_uint8 * n)()
        N.check(N.lib().qs_get_state(self._h, buf, n, self._stream()), "qs_get_state")
        return bytes(buf)

    def set_state(self, blob):
        n = N.lib().qs_state_bytes(self._h)
        if len(blob) < n:
            raise ValueError("state blob too small")
        buf = (ctypes.c_uint8 * n).from_buffer_copy(blob[:n])
        N.check(N.lib().qs_set_state(self._h, buf, n, self._stream()), "qs_set_state")

    # structured views (float32 SoA) for tests / debugging
    def drone_fields(self):
        s = self.state
        return dict(pos=s[N.F_POS:N.F_POS + 3].T, vel=s[N.F_VEL:N.F_VEL + 3].T, rot=s[N.F_ROT:N.F_ROT + 9].T.reshape(-1, 3, 3),
                    omega=s[N.F_OMEGA:N.F_OMEGA + 3].T, rot_damp=s[N.F_ROT_DAMP:N.F_ROT_DAMP + 4].T,
                    cmd_damp=s[N.F_CMD_DAMP:N.F_CMD_DAMP + 4].T, ou=s[N.F_OU:N.F_OU + 4].T, goal=s[N.F_GOAL:N.F_GOAL + 3].T,
                    pid=s[N.F_PID:N.F_PID + 20].T, angle=s[N.F_ANGLE], ang_vel=s[N.F_ANGVEL], heading=s[N.F_HEADING])

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._torch.cuda.synchronize(self.device)
            N.check(N.lib().qs_destroy(self._h), "qs_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _replay_views(torch, ws, rb, rc, E):
    """Zero-copy torch views of the replay state (qs_replay_buffers) inside the torch-owned workspace."""
    slots = rc.keep + rc.buffer_size
    W = int(rb.snap_words)
    base = ws.data_ptr()

    def view(ptr, n, dtype, shape):
        o = int(ptr) - base
        nbytes = n * torch.tensor([], dtype=dtype).element_size()
        return ws[o:o + nbytes].view(dtype).view(*shape)
    return dict(ri=view(rb.ri, N.NR * E, torch.int32, (N.NR, E)), crash=view(rb.crash, E, torch.float64, (E,)),
                hist=view(rb.hist, rc.hist_len * E, torch.float64, (rc.hist_len, E)),
                perm=view(rb.perm, rc.buffer_size * E, torch.int32, (rc.buffer_size, E)),
                nrep=view(rb.nrep, rc.buffer_size * E, torch.int32, (rc.buffer_size, E)),
                store=view(rb.store, E * slots * W, torch.int32, (E, slots, W)), snap_words=W, slots=slots)


def observation_bounds(cfg: QuadSwarmConfig):
    """Observation-space box (QuadrotorSingle.make_observation_space, quadrotor_single.py:278-349 for
    flavor B, quadrotor_single_rewards.py:267-344 for flavor A)."""
    rd = np.array(cfg.room_dims, dtype=np.float64)
    room_range = np.array([rd[0], rd[1], rd[2]])
    vmax, omax = 3.0, 40.0
    if cfg.flavor == "A":
        L = rd[0]
        comp = {"aw": ([-np.pi], [np.pi]), "awdot": ([-omax], [omax]), "cdist": ([0.0], [L / 2]),
                "cdistdot": ([-vmax], [vmax]), "dist": ([-L / 2], [L / 2]), "ndist": ([-L / 2], [L / 2]),
                "distdot": ([-vmax], [vmax]), "angle": ([-np.pi], [np.pi]), "sangle": ([-1.0, -1.0], [1.0, 1.0]),
                "nsangle": ([-1.0, -1.0], [1.0, 1.0]), "angledot": ([-omax], [omax]),
                "rxyz": (list(-room_range), list(room_range)), "rvxyz": ([-2 * vmax] * 3, [2 * vmax] * 3)}
        names = cfg.obs_repr.split("_")
        nb = {"pos_vel": ["rxyz", "rvxyz"], "pos": ["rxyz"], "npos": ["rxyz"], "dist_angle": ["dist", "angle"],
              "dist_sangle": ["dist", "sangle"], "ndist_nsangle": ["dist", "sangle"],
              "dist_angle_heading": ["dist", "angle", "angle"], "dist_sangle_sheading": ["dist", "sangle", "sangle"],
              "none": []}[cfg.neighbor_obs_type]
        names = names + nb * cfg.k_neighbors
        lo = np.concatenate([comp[n][0] for n in names])
        hi = np.concatenate([comp[n][1] for n in names])
        return lo.astype(np.float32), hi.astype(np.float32)
    lo = [-room_range, -vmax * np.ones(3), -np.ones(9), -omax * np.ones(3)]
    hi = [room_range, vmax * np.ones(3), np.ones(9), omax * np.ones(3)]
    if cfg.obs_repr.endswith("floor"):
        lo.append(np.zeros(1)); hi.append(rd[2] * np.ones(1))
    elif cfg.obs_repr.endswith("wall"):
        lo.append(np.zeros(6)); hi.append(5.0 * np.ones(6))
    for _ in range(cfg.k_neighbors):
        lo += [-room_range, -2 * vmax * np.ones(3)]
        hi += [room_range, 2 * vmax * np.ones(3)]
    if cfg.use_obstacles:   # "octmap" (quadrotor_single.py:331)
        lo.append(-10 * np.ones(9)); hi.append(10 * np.ones(9))
    return np.concatenate(lo).astype(np.float32), np.concatenate(hi).astype(np.float32)


def step_blocks(envs, actions, streams):
    """qs_step_blocks: step several env blocks of one device in one C call, block i with actions[i]
    (contiguous fp32 device tensors, checked once by the caller) on streams[i] (torch streams)."""
    n = len(envs)
    hs = (ctypes.c_void_p * n)(*[e._h.value for e in envs])
    acts = (ctypes.c_void_p * n)(*[a.data_ptr() for a in actions])
    sts = (ctypes.c_void_p * n)(*[s.cuda_stream for s in streams])
    N.check(N.lib().qs_step_blocks(hs, n, acts, sts), "qs_step_blocks")
