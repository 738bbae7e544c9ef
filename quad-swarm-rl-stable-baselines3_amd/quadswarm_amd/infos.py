"""Per-step infos of the reference's env step, built on the host from the step kernel's reward components
(buffers.rew_info, config step_infos; rows QS_RI_* of include/quadswarm.h).

Flavor B, every agent, every step: infos[i]["rewards"] = compute_reward_weighted's rew_info
(gym_art/quadrotor_multi/quadrotor_single.py:79-105: the five cost terms and their raw values, negated and scaled
by dt) plus the swarm terms QuadrotorEnvMulti.step adds (quadrotor_multi.py:642-651: rew_quadcol, rew_proximity,
rewraw_quadcol, and with obstacles rew_quadcol_obstacle / rewraw_quadcol_obstacle).
Flavor A, every agent, every step: {"rewards": {}, "goal_dist": |pos - goal|} of the last executed tick
(quadrotor_single_rewards.py:457).
"""
import numpy as np

from . import _native as N

REWARD_KEYS_B = ("rew_main", "rew_pos", "rew_action", "rew_crash", "rew_orient", "rew_spin",
                 "rewraw_main", "rewraw_pos", "rewraw_action", "rewraw_crash", "rewraw_orient", "rewraw_spin",
                 "rew_quadcol", "rew_proximity", "rewraw_quadcol")
REWARD_KEYS_OBST = ("rew_quadcol_obstacle", "rewraw_quadcol_obstacle")
COEFF_KEYS = ("pos", "effort", "crash", "orient", "spin", "quadcol_bin", "quadcol_bin_obst")


def reward_columns_b(comp, coeff, dt, use_obstacles=False):
    """{key: values over the rows} of infos[i]["rewards"] from the reward components comp [QS_NRI, n] (fp32 or
    fp64) and the reward coefficients the step ran with (coeff: COEFF_KEYS).  Same operation order as the
    reference: rew_info[k] = dt * (-(coefficient * raw)) (quadrotor_single.py:79-105)."""
    c = np.asarray(comp, dtype=np.float64)
    dist, eff, crash, orient, spin = (c[k] for k in (N.RI_DIST, N.RI_EFFORT, N.RI_CRASH, N.RI_ORIENT, N.RI_SPIN))
    qc, prox, ob = c[N.RI_QUADCOL], c[N.RI_PROX], c[N.RI_OBST]
    cost_pos = coeff["pos"] * dist
    out = {
        "rew_main": dt * -cost_pos, "rew_pos": dt * -cost_pos,
        "rew_action": dt * -(coeff["effort"] * eff), "rew_crash": dt * -(coeff["crash"] * crash),
        "rew_orient": dt * -(coeff["orient"] * orient), "rew_spin": dt * -(coeff["spin"] * spin),
        "rewraw_main": dt * -dist, "rewraw_pos": dt * -dist, "rewraw_action": dt * -eff,
        "rewraw_crash": dt * -crash, "rewraw_orient": dt * -orient, "rewraw_spin": dt * -spin,
        "rew_quadcol": coeff["quadcol_bin"] * qc, "rew_proximity": prox, "rewraw_quadcol": qc,
    }
    if use_obstacles:
        out["rew_quadcol_obstacle"] = coeff["quadcol_bin_obst"] * ob
        out["rewraw_quadcol_obstacle"] = ob
    return out


def rewards_dict(cols, i):
    """infos[i]["rewards"] of row i from reward_columns_b's columns (python floats, like the reference's)."""
    return {k: float(v[i]) for k, v in cols.items()}


__all__ = ["REWARD_KEYS_B", "REWARD_KEYS_OBST", "COEFF_KEYS", "reward_columns_b", "rewards_dict"]
