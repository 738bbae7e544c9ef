"""Host-side derivation of the quadrotor constants uploaded to the kernels.

Restates, once at env creation:
  * crazyflie_params()                  gym_art/quadrotor_multi/quad_models.py:1-42
  * QuadLink inertia / prop positions   gym_art/quadrotor_multi/inertia.py:182-310
  * QuadrotorDynamics.update_model      gym_art/quadrotor_multi/quadrotor_dynamics.py:106-168
  * the SVD cadence of since_last_svd   quadrotor_dynamics.py:553-558 (float64 accumulation)
Init-only host code: nothing here runs per step.
"""
import math

import numpy as np

GRAV = 9.81
EPS = 1e-6


def crazyflie_params():
    return {
        "geom": {
            "body": {"l": 0.03, "w": 0.03, "h": 0.004, "m": 0.005},
            "payload": {"l": 0.035, "w": 0.02, "h": 0.008, "m": 0.01},
            "arms": {"l": 0.022, "w": 0.005, "h": 0.005, "m": 0.001},
            "motors": {"h": 0.02, "r": 0.0035, "m": 0.0015},
            "propellers": {"h": 0.002, "r": 0.022, "m": 0.00075},
            "motor_pos": {"xyz": [0.065 / 2, 0.065 / 2, 0.0]},
            "arms_pos": {"angle": 45.0, "z": 0.0},
            "payload_pos": {"xy": [0.0, 0.0], "z_sign": 1},
        },
        "damp": {"vel": 0.0, "omega_quadratic": 0.0},
        "noise": {"thrust_noise_ratio": 0.05},
        "motor": {"thrust_to_weight": 1.9, "assymetry": [1.0, 1.0, 1.0, 1.0], "torque_to_thrust": 0.006,
                  "linearity": 1.0, "C_drag": 0.0, "C_roll": 0.0, "damp_time_up": 0.15, "damp_time_down": 0.15},
    }


def _box_I(l, w, h, m):
    return np.diag([m * (h ** 2 + w ** 2) / 12.0, m * (l ** 2 + h ** 2) / 12.0, m * (w ** 2 + l ** 2) / 12.0])


def _cyl_I(h, r, m):
    a = m * (3 * r ** 2 + h ** 2) / 12.0
    return np.diag([a, a, 0.5 * m * r ** 2])


def _translate_diag(I, m, xyz):
    x, y, z = xyz
    return np.array([I[0][0] + m * (y ** 2 + z ** 2), I[1][1] + m * (x ** 2 + z ** 2), I[2][2] + m * (x ** 2 + y ** 2)])


def quad_link(geom):
    """Mass, diagonal inertia about the COM and motor positions (QuadLink, inertia.py:182-310)."""
    arm_angle = math.radians(geom["arms_pos"]["angle"]) or 0.01
    motor_xyz = np.array(geom["motor_pos"]["xyz"], dtype=np.float64)
    body, payload, arms = geom["body"], geom["payload"], dict(geom["arms"])
    delta_y = motor_xyz[1] - body["w"] / 2.0
    if "l" not in arms:
        arms["l"] = delta_y / math.sin(arm_angle)
    arm_xyz = np.array([motor_xyz[0] - delta_y / (2 * math.tan(arm_angle)), motor_xyz[1] - delta_y / 2,
                        geom["arms_pos"]["z"]])
    sign = np.array([[1, -1, -1, 1], [-1, -1, 1, 1], [1.0, 1.0, 1.0, 1.0]])
    motors_coord = sign * motor_xyz[:, None]
    props_coord = motors_coord.copy()
    props_coord[2, :] = props_coord[2, :] + geom["motors"]["h"] / 2.0 + geom["propellers"]["h"]
    arms_coord = sign * arm_xyz[:, None]
    arm_angles = [-arm_angle, arm_angle, -arm_angle, arm_angle]

    links = [(_box_I(body["l"], body["w"], body["h"], body["m"]), body["m"], np.eye(3), np.zeros(3)),
             (_box_I(payload["l"], payload["w"], payload["h"], payload["m"]), payload["m"], np.eye(3),
              np.array(list(geom["payload_pos"]["xy"]) +
                       [np.sign(geom["payload_pos"]["z_sign"]) * (body["h"] + payload["h"]) / 2]))]
    for i in range(4):
        a = arm_angles[i]
        R = np.array([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]])
        links.append((_box_I(arms["l"], arms["w"], arms["h"], arms["m"]), arms["m"], R, arms_coord[:, i]))
    mo, pr = geom["motors"], geom["propellers"]
    for i in range(4):
        links.append((_cyl_I(mo["h"], mo["r"], mo["m"]), mo["m"], np.eye(3), motors_coord[:, i]))
    for i in range(4):
        links.append((_cyl_I(pr["h"], pr["r"], pr["m"]), pr["m"], np.eye(3), props_coord[:, i]))
    masses = [lk[1] for lk in links]
    m_tot = np.sum(masses)
    com = sum(masses[i] * links[i][3] for i in range(len(links))) / m_tot
    I_diag = np.zeros(3)
    for I0, m, R, xyz in links:
        I_rot = R @ I0 @ R.T
        I_diag = I_diag + _translate_diag(I_rot, m, xyz - com)
    prop_pos = np.array([motors_coord[:, i] - com for i in range(4)])
    return float(m_tot), I_diag, prop_pos, motor_xyz


def dynamics_constants(params=None, dt=0.005, thrust_noise_ratio=None):
    """Everything QuadrotorDynamics.update_model derives, as float64."""
    p = params or crazyflie_params()
    mass, inertia, prop_pos, motor_xyz = quad_link(p["geom"])
    mot = p["motor"]
    asym = np.array(mot.get("assymetry", [1.0] * 4), dtype=np.float64)
    asym = asym * 4.0 / np.sum(asym)
    thrust_max = GRAV * mass * mot["thrust_to_weight"] * asym / 4.0
    torque_max = mot["torque_to_thrust"] * thrust_max
    prop_cross = np.cross(prop_pos, [0.0, 0.0, 1.0])
    tnr = p["noise"]["thrust_noise_ratio"] if thrust_noise_ratio is None else thrust_noise_ratio
    return dict(
        mass=mass, inertia=inertia, thrust_max=thrust_max, torque_max=torque_max, prop_cross=prop_cross,
        prop_ccw=np.array([-1.0, 1.0, -1.0, 1.0]), motor_linearity=float(mot["linearity"]),
        motor_tau_up=4 * dt / (mot["damp_time_up"] + EPS), motor_tau_down=4 * dt / (mot["damp_time_down"] + EPS),
        arm=float(np.linalg.norm(motor_xyz[:2])), vel_damp=float(p["damp"]["vel"]),
        damp_omega_quadratic=float(p["damp"]["omega_quadratic"]), ou_sigma=0.2 * tnr,
        C_drag=float(mot["C_drag"]), C_roll=float(mot["C_roll"]))


def svd_every(dt=0.005, limit=0.5):
    """Substeps until since_last_svd (float64 += dt) first exceeds the limit (100 for 0.005 / 0.5)."""
    s, n = 0.0, 0
    while True:
        s += dt
        n += 1
        if s > limit:
            return n
