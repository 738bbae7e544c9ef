"""quadswarm_amd: MI355X-native quadrotor-swarm environment step (HIP/gfx950) behind the reference's
QuadrotorEnvMulti / SB3 VecEnv surface (priban42/quad-swarm-rl-stable-baselines3).

    from quadswarm_amd import QuadSwarmConfig, GpuQuadVecEnv
    venv = GpuQuadVecEnv(QuadSwarmConfig(num_envs=4096, num_agents=8), as_torch=True)
"""
from ._native import QuadSwarmError
from .config import QuadSwarmConfig
from .params import crazyflie_params, dynamics_constants

__all__ = ["QuadSwarmConfig", "QuadSwarmError", "QuadSwarmEnv", "GpuQuadVecEnv", "make_vec_env",
           "crazyflie_params", "dynamics_constants"]


def __getattr__(name):  # torch-dependent pieces load lazily
    if name == "QuadSwarmEnv":
        from .env import QuadSwarmEnv
        return QuadSwarmEnv
    if name in ("GpuQuadVecEnv", "make_vec_env"):
        from . import vec_env
        return getattr(vec_env, name)
    raise AttributeError(name)
