"""Env configuration: the reference's knobs for the flavor-B swarm step, mapped onto qs_config.

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
    apply_collision_force: bool = True
    rew_coeff: dict = field(default_factory=lambda: dict(DEFAULT_REW))
    device: str = "cuda"

    @classmethod
    def from_reference_cfg(cls, cfg, num_envs=None, **over):
        """Adapter for swarm_rl.global_cfg.QuadrotorEnvConfig / SF quads_* namespaces."""
        def g(*names, default=None):
            for n in names:
                if hasattr(cfg, n):
                    return getattr(cfg, n)
            return default
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
            seed=g("seed", default=0) or 0, device=g("device", default="cuda"))
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
        return N.SELF_OBS_DIM[N.OBS_REPR[self.obs_repr]] + 6 * self.k_neighbors

    def validate(self):
        if self.obs_repr not in N.OBS_REPR:
            raise NotImplementedError(f"obs_repr {self.obs_repr!r}: flavor-A representations are not implemented yet")
        if self.neighbor_obs_type not in ("pos_vel", "none"):
            raise NotImplementedError(f"neighbor_obs_type {self.neighbor_obs_type!r} not implemented")
        if self.quads_mode != "static_same_goal":
            raise NotImplementedError(f"quads_mode {self.quads_mode!r} not implemented (static_same_goal only)")
        if not 1 <= self.num_agents <= N.MAX_AGENTS:
            raise ValueError(f"num_agents must be in [1, {N.MAX_AGENTS}]")
        k = self.k_neighbors
        if self.neighbor_obs_type == "pos_vel" and self.num_agents > 1 and not 1 <= k <= self.num_agents - 1:
            raise ValueError("neighbor_visible_num out of range")

    def to_qs_config(self):
        self.validate()
        c = N.QsConfig()
        rc = N.lib().qs_config_default(c, int(self.num_envs), int(self.num_agents))
        N.check(rc, "qs_config_default")
        k = dynamics_constants(crazyflie_params(), dt=self.dt, thrust_noise_ratio=self.thrust_noise_ratio)
        c.obs_repr = N.OBS_REPR[self.obs_repr]
        kn = self.k_neighbors
        c.neighbor_obs = N.NEIGHBOR_POS_VEL if kn > 0 else N.NEIGHBOR_NONE
        c.k_neighbors = kn
        c.ep_len = self.ep_len
        c.sim_steps = self.sim_steps
        c.svd_every = svd_every(self.dt, 0.5)
        c.sense_noise = 0 if self.sense_noise is None else 1
        c.use_downwash = int(bool(self.use_downwash))
        c.apply_collision_force = int(bool(self.apply_collision_force))
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
        return c
