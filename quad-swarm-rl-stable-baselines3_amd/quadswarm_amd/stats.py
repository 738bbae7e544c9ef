"""episode_extra_stats of a finished episode, as the reference's infos carry them.

Flavor B: QuadrotorEnvMulti.step (gym_art/quadrotor_multi/quadrotor_multi.py:739-831) fills
infos[i]["episode_extra_stats"] of every agent when the episode ends; the experience-replay wrapper adds its
"replay/*" values (gym_art/quadrotor_multi/quad_experience_replay.py:124-137).  The step kernel accumulates
the counters on the device and writes one row per drone of a finished env (qs_buffers.estats, the QS_ES_*
columns of include/quadswarm.h); this module turns such a row into the reference's dict -- key names
included ("<scenario>/..." with scenario.name()[9:]).
"""
# QS_ES_* columns (include/quadswarm.h)
ES_COL, ES_ROOM, ES_FLOOR, ES_WALL, ES_CEIL, ES_COL_SETTLE, ES_COL_FINAL = range(7)
ES_OCOL, ES_OCOL_SETTLE, ES_O35, ES_O5 = 7, 8, 9, 10
ES_SUCCESS, ES_DEADLOCK, ES_COLRATE, ES_NCOLRATE, ES_OCOLRATE, ES_SCEN, ES_D1, ES_D3, ES_D5, ES_REPLAY = range(11, 21)
NES = 24

# scenario id of a row -> the reference's scenario class name minus "Scenario_": QUADS_MODE_LIST order
# (scenarios/utils.py:7-10) + run_away for the goal scenarios, 16 + mode for the obstacle ones (19-21: the maps'
# dynamic scenarios, qs_flavor_b.h obst_stats_id)
SCENARIO_NAMES = {0: "static_same_goal", 1: "static_diff_goal", 2: "ep_lissajous3D", 3: "ep_rand_bezier",
                  4: "dynamic_same_goal", 5: "dynamic_diff_goal", 6: "dynamic_formations", 7: "swap_goals",
                  8: "swarm_vs_swarm", 9: "run_away", 16: "o_random", 17: "o_static_same_goal",
                  18: "dynamic_repulsive",   # flavor A's target-chasing scenario
                  19: "o_swap_goals", 20: "o_ep_rand_bezier", 21: "o_dynamic_same_goal"}


def episode_extra_stats(row, use_obstacles=False):
    """The reference's infos[i]["episode_extra_stats"] dict of agent i from its stats row (sequence of at least
    21 numbers: the QS_ES_* columns).  Counts are ints, rates and distances floats."""
    r = [float(x) for x in row]
    if r[ES_REPLAY] != 0:   # saved_in_replay_buffer: a replayed episode reports only these (:742-746)
        return {"num_collisions_replay": int(r[ES_COL]), "num_collisions_obst_replay": int(r[ES_OCOL])}
    sc = SCENARIO_NAMES.get(int(r[ES_SCEN]), "static_same_goal")
    d = {
        "num_collisions": int(r[ES_COL]),
        "num_collisions_with_room": int(r[ES_ROOM]),
        "num_collisions_with_floor": int(r[ES_FLOOR]),
        "num_collisions_with_wall": int(r[ES_WALL]),
        "num_collisions_with_ceiling": int(r[ES_CEIL]),
        "num_collisions_after_settle": int(r[ES_COL_SETTLE]),
        f"{sc}/num_collisions": int(r[ES_COL_SETTLE]),
        "num_collisions_final_5_s": int(r[ES_COL_FINAL]),
        f"{sc}/num_collisions_final_5_s": int(r[ES_COL_FINAL]),
        "distance_to_goal_1s": r[ES_D1],
        "distance_to_goal_3s": r[ES_D3],
        "distance_to_goal_5s": r[ES_D5],
        f"{sc}/distance_to_goal_1s": r[ES_D1],
        f"{sc}/distance_to_goal_3s": r[ES_D3],
        f"{sc}/distance_to_goal_5s": r[ES_D5],
    }
    if use_obstacles:
        d.update({"num_collisions_obst_quad": int(r[ES_OCOL]),
                  "num_collisions_obst_quad_after_settle": int(r[ES_OCOL_SETTLE]),
                  f"{sc}/num_collisions_obst": int(r[ES_OCOL]),
                  "num_collisions_obst_quad_3_5": int(r[ES_O35]),
                  f"{sc}/num_collisions_obst_quad_3_5": int(r[ES_O35]),
                  "num_collisions_obst_quad_5": int(r[ES_O5]),
                  f"{sc}/num_collisions_obst_quad_5": int(r[ES_O5])})
    for name, col in (("agent_success_rate", ES_SUCCESS), ("agent_deadlock_rate", ES_DEADLOCK),
                      ("agent_col_rate", ES_COLRATE), ("agent_neighbor_col_rate", ES_NCOLRATE),
                      ("agent_obst_col_rate", ES_OCOLRATE)):
        d[f"metric/{name}"] = r[col]
        d[f"{sc}/{name}"] = r[col]
    return d
