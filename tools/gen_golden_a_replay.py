#!/usr/bin/env python
"""What the reference does with flavor A + the experience-replay wrapper.  TEST INFRASTRUCTURE, dev
container only (imports the reference through tools/refshim.py like the other generators).

    python tools/gen_golden_a_replay.py     # writes tests/golden/a_replay_outcome.json
                                            # and tests/golden/quadrotor_env_config.json

The second fixture is the field set and default values of the reference's own `QuadrotorEnvConfig`
(`swarm_rl/global_cfg.py`), which `QuadSwarmConfig.from_reference_cfg` adapts.

sb_train builds `ExperienceReplayWrapper(QuadrotorEnvMulti(cfg), 0.5, ...)` when `cfg.use_replay_buffer`
(`swarm_rl/env_wrappers/sb3_quad_env.py:43-45`) around the flavor-A env (`quadrotor_multi_rewards.py`) and
runs it in the SubprocVecEnvCustom worker.  This script drives exactly that stack: SB3QuadrotorEnv.step's
5-tuple (`sb3_quad_env.py:56-59`) and the worker's done branch (`subproc_vec_env_custom.py:33-47`, restated
below because stable_baselines3 is not importable here) until the first episode end, and records what
happens there.  The fixture is plain JSON (outcome strings and numbers), no reference source.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the shims)
import gen_golden_a as GA  # noqa: E402

from gym_art.quadrotor_multi.quad_experience_replay import ExperienceReplayWrapper  # noqa: E402


def probe(n, seed, steps=80):
    np.random.seed(seed)
    env = GA.make_env_A(n, seed=seed, ntype="dist_angle", repr_="cdist_cdistdot_dist_distdot_angle_angledot",
                        ep_time=2.0, capture=0.01)
    env.use_replay_buffer = True          # cfg.use_replay_buffer (quadrotor_multi_rewards.py:153)
    cfg = env.cfg
    w = ExperienceReplayWrapper(env, 0.5, cfg.obst_density, cfg.obst_size, False, False, False, 0, 1, 0.1, 1.0)
    obs, info = w.reset()                 # SB3QuadrotorEnv.reset (sb3_quad_env.py:52-55)
    out = {"n": n, "seed": seed, "reset_obs_type": type(obs).__name__}
    act_rng = np.random.default_rng(seed + 300)
    for t in range(steps):
        a = act_rng.uniform(-1.0, 1.0, (n, 2))
        try:
            obs, reward, term, info = w.step(a)
        except Exception as e:  # noqa: BLE001  (the reference's own failure is the recorded outcome)
            out["step_error"] = f"{type(e).__name__}: {e}"
            out["step_error_at"] = t
            break
        done = np.array(term) | np.array(term)
        if any(done):
            out["first_done_step"] = t
            out["obs_type_at_done"] = type(obs).__name__
            out["obs_len_at_done"] = len(obs)
            try:   # the worker's done branch: terminal_observation = observation[i] for every agent's info
                for i in range(len(info)):
                    info[i]["terminal_observation"] = obs[i]
                out["worker"] = "ok"
            except Exception as e:  # noqa: BLE001
                out["worker"] = f"{type(e).__name__}: {e}"
                out["failed_at_agent"] = i
            out["replay_keys"] = sorted(k for k in info[0]["episode_extra_stats"] if k.startswith("replay/"))
            break
    return out


def env_config_fields():
    import dataclasses
    from swarm_rl.global_cfg import QuadrotorEnvConfig
    c = QuadrotorEnvConfig()
    out = {}
    for f in dataclasses.fields(c):
        v = getattr(c, f.name)
        if isinstance(v, np.ndarray):
            v = v.tolist()
        if isinstance(v, tuple):
            v = list(v)
        try:
            json.dumps(v)
        except TypeError:
            v = repr(v)
        out[f.name] = v
    return out


def main():
    with open(os.path.join(G.OUT, "quadrotor_env_config.json"), "w") as f:
        json.dump(env_config_fields(), f, indent=1, sort_keys=True)
    res = {"stack": "ExperienceReplayWrapper(flavor-A QuadrotorEnvMulti) + SubprocVecEnvCustom worker",
           "cases": [probe(8, 51), probe(4, 52), probe(2, 53)]}
    path = os.path.join(G.OUT, "a_replay_outcome.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
