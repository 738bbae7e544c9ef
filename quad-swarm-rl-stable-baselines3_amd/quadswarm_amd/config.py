"""Env configuration: the reference's knobs for the swarm step (flavors B and A), mapped onto qs_config.

flavor "B": gym_art.quadrotor_multi.quadrotor_multi.QuadrotorEnvMulti (raw motor commands, shaped rewards).
flavor "A": gym_art.quadrotor_multi.quadrotor_multi_rewards.QuadrotorEnvMulti, the env swarm_rl/sb_train.py
            builds (sb3_quad_env.py:34-41): PID pre-controller, heading-rate action, capture reward.

Field names follow the reference's own configs so existing configs drop in:
  * swarm_rl/global_cfg.py:7-190 (QuadrotorEnvConfig, used by sb_train)
  * swarm_rl/env_wrappers/quadrotor_params.py:15-122 (quads_* CLI of the SF path)
  * swarm_rl/env_wrappers/quad_utils.py:20-68 (what make_quadrotor_env_multi passes to QuadrotorEnvMulti)
"""
from dataclasses import dataclass, field
from typing import Optional

from . import _native as N
from .params import crazyflie_params, dynamics_constants, svd_every

DEFAULT_REW = dict(pos=1.0, effort=0.05, crash=1.0, orient=1.0, spin=0.1,
                   quadcol_bin=5.0, quadcol_bin_smooth_max=10.0)


@dataclass
class QuadSwarmConfig:
    num_envs: int = 4096
    num_agents: int = 8
    obs_repr: str = "xyz_vxyz_R_omega"
    episode_duration: float = 15.0            # quads_episode_duration
    neighbor_visible_num: int = 6             # -1 = all (no sorting)
    neighbor_obs_type: str = "pos_vel"
    collision_hitbox_radius: float = 2.0      # x arm
    collision_falloff_radius: float = 4.0     # x arm
    collision_reward: float = 5.0             # quadcol_bin
    collision_smooth_max_penalty: float = 10.0
    use_downwash: bool = False
    quads_mode: str = "static_same_goal"
    room_dims: tuple = (10.0, 10.0, 10.0)
    sense_noise: Optional[str] = "default"    # None -> SensorNoise(bypass=True)
    thrust_noise_ratio: float = 0.05
    sim_freq: float = 200.0
    sim_steps: int = 2
    seed: int = 0
    drone_id_offset: int = 0                  # global id of this shard's first drone (multi-GPU)
    specialize: bool = True                   # qs_specialize: hipRTC kernels with this config's constants baked in
    apply_collision_force: bool = True
    rew_coeff: dict = field(default_factory=lambda: dict(DEFAULT_REW))
    device: str = "cuda"
    # ---- flavor A (swarm_rl/global_cfg.py:14-40) ----
    flavor: str = "B"
    initial_capture_radius: float = 3.0
    focal_length_cam: float = 0.035
    n_cameras: int = 3
    neighbour_size_cam: float = 0.2
    pixel_noise_cam: float = 3.0
    ticks_per_step: int = 8                   # QuadrotorSingle._step calls per env step (:636)
    # ---- obstacles (flavor B; quadrotor_params.py quads_obst_*, quad_obstacle_baseline.py) ----
    use_obstacles: bool = False
    obst_density: float = 0.2
    obst_size: float = 0.6
    obst_spawn_area: tuple = (8, 8)
    obst_collision_reward: float = 5.0        # quadcol_bin_obst
    # ---- experience replay (quad_utils.py:34, 68-71: on when > 0; the reference's swarm runs use 0.75) ----
    replay_buffer_sample_prob: float = 0.0
    # ---- obstacle domain randomisation (quadrotor_params.py:62-72 / global_cfg.py:85-91), applied by the replay
    # wrapper's reset (quad_experience_replay.py:76-87, 106-118, 206-214): only with replay on, as the
    # reference only builds the wrapper then (quad_utils.py:68-71) ----
    domain_random: bool = False
    obst_density_random: bool = False
    obst_density_min: float = 0.05
    obst_density_max: float = 0.2
    obst_size_random: bool = False
    obst_size_min: float = 0.3
    obst_size_max: float = 0.6
    # ---- episode_extra_stats (flavor B, quadrotor_multi.py:739-831): the reference always keeps them; the
    # step kernels do so when on (infos of finished envs, GpuQuadVecEnv) ----
    episode_stats: bool = True
    # ---- per-step infos (quadrotor_single.py:79-105, quadrotor_multi.py:642-651; flavor A
    # quadrotor_single_rewards.py:457): the step writes each drone's reward components (buffers.rew_info), from
    # which GpuQuadVecEnv builds infos[i]["rewards"] / infos[i]["goal_dist"].  Off for the raw env (the bench's
    # step does not pay for it); GpuQuadVecEnv turns it on (infos=True) ----
    step_infos: bool = False

    @classmethod
    def c4(cls, num_envs=4096, num_agents=8, **over):
        """8 drones + obstacles (8x8 m area, density 0.2 -> 12 pillars of 0.6 m),
        xyz_vxyz_R_omega_floor + pos_vel k=2 + 9 SDF = 40 obs, downwash, quads_mode mix
        (o_random / o_static_same_goal), 15 s episodes (swarm_rl/runs/obstacles/quad_obstacle_baseline.py)."""
        c = cls(num_envs=num_envs, num_agents=num_agents, obs_repr="xyz_vxyz_R_omega_floor", neighbor_visible_num=2,
                neighbor_obs_type="pos_vel", use_obstacles=True, use_downwash=True, quads_mode="mix",
                collision_smooth_max_penalty=4.0)
        for k, v in over.items():
            setattr(c, k, v)
        return c

    @classmethod
    def sb_train(cls, num_envs=4096, num_agents=8, **over):
        """Flavor A exactly as swarm_rl/sb_train.py trains it (global_cfg.py defaults + parameter_sweep
        sb_train.py:111-139): dynamic_repulsive, 15x15x3 room, 30 s episodes, cdist..sangle self obs,
        camera neighbours (ndist_nsangle) of all N-1 drones, pixel noise 0."""
        c = cls(num_envs=num_envs, num_agents=num_agents, flavor="A",
                obs_repr="cdist_cdistdot_dist_distdot_sangle_angledot", episode_duration=30.0,
                neighbor_visible_num=-1, neighbor_obs_type="ndist_nsangle", quads_mode="dynamic_repulsive",
                room_dims=(15.0, 15.0, 3.0), pixel_noise_cam=0.0, apply_collision_force=False)
        for k, v in over.items():
            setattr(c, k, v)
        return c

    @classmethod
    def from_reference_cfg(cls, cfg, num_envs=None, flavor=None, **over):
        """Adapter for swarm_rl.global_cfg.QuadrotorEnvConfig / SF quads_* namespaces.  A config with
        dim_mode '2D_horizontal' (global_cfg.py:41, what sb_train builds) maps to flavor A."""
        def g(*names, default=None):
            for n in names:
                if hasattr(cfg, n):
                    return getattr(cfg, n)
            return default
        if flavor is None:
            flavor = "A" if g("dim_mode", default="3D") == "2D_horizontal" else "B"
        c = cls(
            num_envs=num_envs or g("num_envs", default=1),
            num_agents=g("num_agents", "quads_num_agents", default=8),
            obs_repr=g("obs_repr", "quads_obs_repr", default="xyz_vxyz_R_omega"),
            episode_duration=g("episode_duration", "quads_episode_duration", default=15.0),
            neighbor_visible_num=g("neighbor_visible_num", "quads_neighbor_visible_num", default=-1),
            neighbor_obs_type=g("neighbor_obs_type", "quads_neighbor_obs_type", default="pos_vel"),
            collision_hitbox_radius=g("collision_hitbox_radius", "quads_collision_hitbox_radius", default=2.0),
            collision_falloff_radius=g("collision_falloff_radius", "quads_collision_falloff_radius", default=4.0),
            collision_reward=g("collision_reward", "quads_collision_reward", default=5.0),
            collision_smooth_max_penalty=g("collision_smooth_max_penalty", "quads_collision_smooth_max_penalty",
                                           default=10.0),
            use_downwash=g("use_downwash", "quads_use_downwash", default=False),
            quads_mode=g("quads_mode", default="static_same_goal"),
            room_dims=tuple(g("room_dims", "quads_room_dims", default=(10.0, 10.0, 10.0))),
            sense_noise=g("sense_noise", default="default"),
            thrust_noise_ratio=g("thrust_noise_ratio", default=0.05),
            sim_freq=g("sim_freq", default=200.0), sim_steps=g("sim_steps", default=2),
            seed=g("seed", default=0) or 0, device=g("device", default="cuda"), flavor=flavor,
            use_obstacles=bool(g("use_obstacles", "quads_use_obstacles", default=False)),
            obst_density=g("obst_density", "quads_obst_density", default=0.2),
            obst_size=g("obst_size", "quads_obst_size", default=0.6),
            obst_spawn_area=tuple(g("obst_spawn_area", "quads_obst_spawn_area", default=(8, 8))),
            obst_collision_reward=g("obst_collision_reward", "quads_obst_collision_reward", default=5.0),
            replay_buffer_sample_prob=g("replay_buffer_sample_prob", default=0.0) or 0.0,
            domain_random=bool(g("domain_random", "quads_domain_random", default=False)),
            obst_density_random=bool(g("obst_density_random", "quads_obst_density_random", default=False)),
            obst_density_min=g("obst_density_min", "quads_obst_density_min", default=0.05),
            obst_density_max=g("obst_density_max", "quads_obst_density_max", default=0.2),
            obst_size_random=bool(g("obst_size_random", "quads_obst_size_random", default=False)),
            obst_size_min=g("obst_size_min", "quads_obst_size_min", default=0.3),
            obst_size_max=g("obst_size_max", "quads_obst_size_max", default=0.6))
        if flavor == "A":
            # sb_train wraps the env in ExperienceReplayWrapper(env, 0.5, ...) when cfg.use_replay_buffer
            # (sb3_quad_env.py:43-45)
            # only; its QuadrotorEnvConfig's replay_buffer_sample_prob (0.75) is the SF runs' knob, unused here
            c.replay_buffer_sample_prob = 0.5 if g("use_replay_buffer", default=False) else 0.0
            # quadrotor_multi_rewards builds its dynamics from cfg.dynamics_change only (the
            # thrust_noise_ratio it computes at :46-49 is never used), default Crazyflie noise 0.05
            dc = g("dynamics_change", default=None) or {}
            c.thrust_noise_ratio = (dc.get("noise") or {}).get("thrust_noise_ratio", 0.05)
            c.apply_collision_force = False   # quadrotor_multi_rewards.py:203
            ic = g("initial_capture_radius", default=None)
            c.initial_capture_radius = 0.2 if ic is None else ic   # :205-208
            for n in ("focal_length_cam", "n_cameras", "neighbour_size_cam", "pixel_noise_cam"):
                if hasattr(cfg, n):
                    setattr(c, n, getattr(cfg, n))
        for k, v in over.items():
            setattr(c, k, v)
        return c

    # ---- derived ----
    @property
    def dt(self):
        return 1.0 / self.sim_freq

    @property
    def ep_len(self):
        return int(self.episode_duration / (self.dt * self.sim_steps))   # quadrotor_single.py:158

    @property
    def k_neighbors(self):
        if self.neighbor_obs_type == "none" or self.num_agents == 1:
            return 0
        return self.num_agents - 1 if self.neighbor_visible_num == -1 else self.neighbor_visible_num

    @property
    def obs_dim(self):
        return N.SELF_OBS_DIM[N.OBS_REPR[self.obs_repr]] + N.NEIGHBOR_DIM[N.NEIGHBOR[self.neighbor_obs_type]] * \
            self.k_neighbors + (9 if self.use_obstacles else 0)

    @property
    def num_obstacles(self):   # quadrotor_multi.py:138
        return int(self.obst_density * self.obst_spawn_area[0] * self.obst_spawn_area[1])

    @property
    def domain_random_active(self):
        return bool(self.use_obstacles and self.replay_buffer_sample_prob > 0 and self.domain_random
                    and (self.obst_density_random or self.obst_size_random))

    def domain_random_tables(self):
        """(densities, pillar counts, sizes) of the replay wrapper's choice lists: np.arange(min, max, 0.05) /
        np.arange(min, max, 0.1) (quad_experience_replay.py:82, 86), count = int(area^2 * density)
        (quadrotor_multi.py:414).  A 0.0 choice is falsy at quadrotor_multi.py:443-446, i.e. the env keeps its
        current value: count -1 / size 0.0.  Empty lists when that randomisation is off."""
        import numpy as np
        dens = np.arange(self.obst_density_min, self.obst_density_max, 0.05) if self.obst_density_random else np.zeros(0)
        sizes = np.arange(self.obst_size_min, self.obst_size_max, 0.1) if self.obst_size_random else np.zeros(0)
        cells = int(self.obst_spawn_area[0]) * int(self.obst_spawn_area[1])
        counts = [int(cells * d) if d else -1 for d in dens]
        return dens, counts, sizes

    @property
    def max_obstacles(self):
        """Pillar slots per env: the configured count or the largest domain-randomisation choice."""
        if not self.domain_random_active:
            return self.num_obstacles
        return max([self.num_obstacles] + self.domain_random_tables()[1])

    @property
    def scenario_id(self):
        if self.use_obstacles:
            return N.SCENARIO_OBST[self.quads_mode]
        if self.flavor == "B" or self.quads_mode not in N.SCENARIO:
            return N.SCENARIO_B[self.quads_mode]   # goal scenarios (create_scenario) of either flavor
        return N.SCENARIO[self.quads_mode]

    @property
    def act_dim(self):
        return 2 if self.flavor == "A" else 4

    def validate(self):
        if self.flavor not in ("A", "B"):
            raise ValueError(f"flavor must be 'A' or 'B', got {self.flavor!r}")
        if self.obs_repr not in N.OBS_REPR:
            raise NotImplementedError(f"obs_repr {self.obs_repr!r} not implemented")
        rid = N.OBS_REPR[self.obs_repr]
        if rid not in (N.OBS_REPR_A if self.flavor == "A" else N.OBS_REPR_B):
            raise ValueError(f"obs_repr {self.obs_repr!r} does not belong to flavor {self.flavor}")
        if self.neighbor_obs_type not in N.NEIGHBOR:
            raise NotImplementedError(f"neighbor_obs_type {self.neighbor_obs_type!r} not implemented")
        if self.flavor == "B" and self.neighbor_obs_type not in ("pos_vel", "none"):
            raise NotImplementedError(f"flavor B implements neighbor_obs_type pos_vel / none")
        if self.flavor == "B" and not self.use_obstacles and self.quads_mode not in N.SCENARIO_B:
            raise NotImplementedError(f"quads_mode {self.quads_mode!r} not implemented for flavor B "
                                      f"({', '.join(N.SCENARIO_B)})")
        if self.flavor == "B" and self.quads_mode == "run_away" and self.num_agents < 2:
            raise ValueError("run_away needs at least 2 drones")
        if self.use_obstacles:
            if self.flavor != "B":
                raise NotImplementedError("obstacles are implemented for flavor B")
            if self.quads_mode not in N.SCENARIO_OBST:
                raise NotImplementedError(f"quads_mode {self.quads_mode!r} with obstacles ({', '.join(N.SCENARIO_OBST)})")
            a = self.obst_spawn_area
            if a[0] != a[1] or int(a[0]) != a[0] or not 1 <= a[0] <= 8:
                raise NotImplementedError("obst_spawn_area must be a square of 1..8 cells")
            if self.domain_random_active:
                dens, counts, sizes = self.domain_random_tables()
                if len(dens) > N.MAX_DR_CHOICES or len(sizes) > N.MAX_DR_CHOICES:
                    raise NotImplementedError(f"at most {N.MAX_DR_CHOICES} domain-randomisation choices per list")
                if any(c == 0 for c in counts):
                    raise ValueError("a density choice gives 0 pillars (the reference's obstacle arrays break)")
        if self.flavor == "A":
            if self.quads_mode not in ("dynamic_repulsive", "static_same_goal") and self.quads_mode not in N.SCENARIO_B:
                raise NotImplementedError(f"quads_mode {self.quads_mode!r} not implemented for flavor A "
                                          "(dynamic_repulsive or a goal scenario of create_scenario)")
        if self.replay_buffer_sample_prob > 0 and self.flavor != "B":
            # The reference's flavor-A replay stack (sb3_quad_env.py:43-45) cannot step: its step reads
            # infos[0]["rewards"]["rew_crash"] while the replay buffer is inactive (quadrotor_multi_rewards.py:
            # 871-872), and flavor A's per-drone info carries an empty "rewards" dict (quadrotor_single_rewards.py:
            # 457), so the first step raises KeyError (tests/golden/a_replay_outcome.json, from the reference
            # itself).  There is no reference behaviour to reproduce, so the build refuses it the same way.
            raise KeyError("rew_crash: the reference's flavor-A env cannot run the experience-replay wrapper "
                           "(quadrotor_multi_rewards.py:872 reads a reward the flavor-A step does not report)")
        if not 0.0 <= self.replay_buffer_sample_prob <= 1.0:
            raise ValueError("replay_buffer_sample_prob must be in [0, 1]")
        if not 1 <= self.num_agents <= N.MAX_AGENTS:
            raise ValueError(f"num_agents must be in [1, {N.MAX_AGENTS}]")
        k = self.k_neighbors
        if self.neighbor_obs_type != "none" and self.num_agents > 1 and not 1 <= k <= self.num_agents - 1:
            raise ValueError("neighbor_visible_num out of range")
        # qs_step.hip validate: flavor-A envs of more than 64 drones keep their k nearest in registers
        if self.flavor == "A" and self.num_agents > 64 and self.neighbor_obs_type != "none" and k > N.A_KMAX:
            raise ValueError(f"flavor A with more than 64 drones: neighbor_visible_num must be <= {N.A_KMAX}")

    def to_qs_config(self):
        self.validate()
        c = N.QsConfig()
        rc = N.lib().qs_config_default(c, int(self.num_envs), int(self.num_agents))
        N.check(rc, "qs_config_default")
        k = dynamics_constants(crazyflie_params(), dt=self.dt, thrust_noise_ratio=self.thrust_noise_ratio)
        c.flavor = N.FLAVOR_A if self.flavor == "A" else N.FLAVOR_B
        c.obs_repr = N.OBS_REPR[self.obs_repr]
        kn = self.k_neighbors
        c.neighbor_obs = N.NEIGHBOR[self.neighbor_obs_type] if kn > 0 else N.NEIGHBOR_NONE
        c.k_neighbors = kn
        c.scenario = self.scenario_id
        c.ticks_per_step = int(self.ticks_per_step)
        c.capture_radius = float(self.initial_capture_radius)
        c.cam_size, c.cam_focal, c.cam_px_noise = self.neighbour_size_cam, self.focal_length_cam, self.pixel_noise_cam
        c.n_cameras = int(self.n_cameras)
        c.ep_len = self.ep_len
        c.sim_steps = self.sim_steps
        c.svd_every = svd_every(self.dt, 0.5)
        c.sense_noise = 0 if self.sense_noise is None else 1
        c.use_downwash = int(bool(self.use_downwash))
        c.apply_collision_force = int(bool(self.apply_collision_force)) if self.flavor == "B" else 0
        c.seed = int(self.seed) & 0xFFFFFFFF
        c.drone_id_offset = int(self.drone_id_offset)
        c.dt = self.dt
        c.control_dt = self.dt * self.sim_steps
        c.mass = k["mass"]
        for i in range(3):
            c.inertia[i] = k["inertia"][i]
        for j in range(4):
            c.thrust_max[j] = k["thrust_max"][j]
            c.torque_max[j] = k["torque_max"][j]
            c.prop_ccw[j] = k["prop_ccw"][j]
            for a in range(3):
                c.prop_cross[j][a] = k["prop_cross"][j][a]
        c.motor_tau_up, c.motor_tau_down = k["motor_tau_up"], k["motor_tau_down"]
        c.motor_linearity = k["motor_linearity"]
        c.arm = k["arm"]
        c.vel_damp, c.damp_omega_quadratic = k["vel_damp"], k["damp_omega_quadratic"]
        c.ou_sigma = k["ou_sigma"]
        rd = self.room_dims
        lo, hi = (-rd[0] / 2.0, -rd[1] / 2.0, 0.0), (rd[0] / 2.0, rd[1] / 2.0, float(rd[2]))
        for i in range(3):
            c.room_lo[i], c.room_hi[i] = lo[i], hi[i]
        c.collision_threshold = self.collision_hitbox_radius * k["arm"]
        c.collision_falloff_threshold = self.collision_falloff_radius * k["arm"]
        r = self.rew_coeff
        c.rew_pos, c.rew_effort, c.rew_crash = r.get("pos", 1.0), r.get("effort", 0.05), r.get("crash", 1.0)
        c.rew_orient, c.rew_spin = r.get("orient", 1.0), r.get("spin", 0.1)
        c.rew_quadcol_bin = self.collision_reward
        c.rew_quadcol_smooth_max = self.collision_smooth_max_penalty
        if self.use_obstacles:
            c.use_obstacles = 1
            c.num_obstacles = self.num_obstacles
            c.obst_area = int(self.obst_spawn_area[0])
            c.obst_size = self.obst_size
            c.rew_quadcol_bin_obst = self.obst_collision_reward
            c.spawn_box = 0.1   # QuadrotorSingle.box with obstacles (quadrotor_single.py:238-241)
            if self.domain_random_active:
                dens, counts, sizes = self.domain_random_tables()
                c.dr_num_counts = len(counts)
                for i, v in enumerate(counts):
                    c.dr_counts[i] = v
                c.dr_num_sizes = len(sizes)
                for i, v in enumerate(sizes):
                    c.dr_sizes[i] = float(v)
        c.episode_stats = 1 if self.episode_stats else 0
        c.step_infos = 1 if self.step_infos else 0
        return c
