"""The reference's parameter surfaces.

* ROS node parameters (config/nmpc_nav_control.yaml, parsed by NMPCNavControlROS::readParam,
  src/nmpc_nav_control/NMPCNavControlROS.cpp:44-302): steering geometry, control_freq, wheel geometry,
  limits and the diagonal weights. ``from_ros_params`` validates exactly like readParam (same messages)
  and returns the solver parameters the wrapper constructors would set.
* Codegen parameters (config/nmpc_nav_control_acados_models.yaml, read by scripts/*/common.py:4-21):
  tf_ini and freq fix the horizon N = ceil(tf_ini * freq) and the solver time step.
"""
import math

import yaml

from ._lib import MODEL_IDS, default_params

GEOMETRIES = {"diff": "diff", "omni4": "omni4", "tric": "tric"}  # kDiffStr / kOmni4Str / kTricStr


def load_yaml(path):
    with open(path) as f:
        return yaml.safe_load(f)


def horizon_from_codegen(params):
    """scripts/diff/common.py:5-9: dt = 1/freq, N = ceil(tf_ini/dt)."""
    dt = 1.0 / params["freq"]
    N = int(math.ceil(params["tf_ini"] / dt))
    return N, dt


def _numeric_array(P, key, n):
    val = P.get(key)
    msg = f"Parameter '{key}' must be an array of {n} numeric values."
    if not isinstance(val, list) or len(val) != n:
        raise RuntimeError(msg)
    out = []
    for v in val:
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            raise RuntimeError(msg)
        out.append(float(v))
    return out


def _require(P, keys, geometry):
    if any(k not in P for k in keys):
        raise RuntimeError(f"The steering geometry {geometry} requires the definition of the following "
                           f"parameters: {', '.join(keys)}")


def from_ros_params(P, N=None, codegen=None):
    """Build (model, nmpc_model_params) from a ROS parameter dict (readParam, NMPCNavControlROS.cpp:44-302).

    N / solver dt come from the codegen dict when given (its `<geometry>_params` block), else N stays
    as passed (default 80, the shipped codegen horizon) and the solver dt = 1/control_freq."""
    if "steering_geometry" not in P:
        raise RuntimeError("The node nmpc_nav_control requires the definition of the steering_geometry parameter")
    geometry = P["steering_geometry"]
    if geometry not in GEOMETRIES:
        raise RuntimeError("Invalid steering_geometry (check documentation for supported ones)")
    control_freq = int(P.get("control_freq", 40))
    dt_ctrl = 1.0 / float(control_freq)
    solver_dt = dt_ctrl
    if codegen is not None and f"{geometry}_params" in codegen:
        N, solver_dt = horizon_from_codegen(codegen[f"{geometry}_params"])
    N = 80 if N is None else int(N)
    prm = default_params(geometry, N)
    prm.model = MODEL_IDS[geometry]
    prm.dt = solver_dt
    prm.dt_ctrl = dt_ctrl
    from ._lib import lib
    if geometry == "omni4":
        _require(P, ["rob_dist_between_front_back_wh", "rob_dist_between_left_right_wh", "rob_wh_vel_time_const",
                     "rob_wh_max_vel", "rob_wh_max_ace"], geometry)
        Q = _numeric_array(P, "cost_matrix_weights_state_diag", 11)
        R = _numeric_array(P, "cost_matrix_weights_input_diag", 4)
        prm.p[0] = float(P["rob_dist_between_front_back_wh"]) + float(P["rob_dist_between_left_right_wh"])
        prm.p[1] = float(P["rob_wh_vel_time_const"])
        lib().nmpc_model_params_set_limits(prm, float(P["rob_wh_max_vel"]), float(P["rob_wh_max_ace"]), 0, 0, 0)
        W = Q + R
    elif geometry == "diff":
        _require(P, ["rob_dist_between_wh", "rob_wh_vel_time_const", "rob_wh_max_vel", "rob_wh_max_ace",
                     "cost_matrix_weights_state_diag", "cost_matrix_weights_input_diag"], geometry)
        Q = _numeric_array(P, "cost_matrix_weights_state_diag", 7)
        R = _numeric_array(P, "cost_matrix_weights_input_diag", 2)
        prm.p[0] = float(P["rob_dist_between_wh"])
        prm.p[1] = float(P["rob_wh_vel_time_const"])
        lib().nmpc_model_params_set_limits(prm, float(P["rob_wh_max_vel"]), float(P["rob_wh_max_ace"]), 0, 0, 0)
        W = Q + R
    else:
        _require(P, ["steering_wheel_frame_id", "rob_dist_between_steering_back_wh", "rob_wh_vel_time_const",
                     "rob_steer_wh_angle_time_const", "rob_wh_max_vel", "rob_wh_max_ace", "rob_steer_wh_min_angle",
                     "rob_steer_wh_max_angle", "rob_steer_wh_max_angle_var"], geometry)
        Q = _numeric_array(P, "cost_matrix_weights_state_diag", 7)
        R = _numeric_array(P, "cost_matrix_weights_input_diag", 2)
        prm.p[0] = float(P["rob_dist_between_steering_back_wh"])
        prm.p[1] = float(P["rob_wh_vel_time_const"])
        prm.p[2] = float(P["rob_steer_wh_angle_time_const"])
        d = math.pi / 180.0
        lib().nmpc_model_params_set_limits(prm, float(P["rob_wh_max_vel"]), float(P["rob_wh_max_ace"]),
                                           float(P["rob_steer_wh_min_angle"]) * d,
                                           float(P["rob_steer_wh_max_angle"]) * d,
                                           float(P["rob_steer_wh_max_angle_var"]) * d)
        W = Q + R
    for i, w in enumerate(W):
        prm.W[i] = w
    for i, w in enumerate(Q):
        prm.W_e[i] = w  # constructors initialise W_e with Q_diag (NMPCNavControlDiff.cpp:39-41)
    return geometry, prm
