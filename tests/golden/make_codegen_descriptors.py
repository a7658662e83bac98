"""Generate tests/golden/codegen_descriptors.json: the reference's own codegen parameter loader
(scripts/{diff,omni4,tric}/common.py:load_parameters, numpy only) evaluated on the shipped codegen yaml
(config/nmpc_nav_control_acados_models.yaml) and on variations of its horizon / rate / bound keys.

Run in the build container, where /root/reference exists (the GPU box never runs this):
    python tests/golden/make_codegen_descriptors.py
The fixture holds inputs and outputs only; tests/test_codegen.py pins tools/generate_solver_libs.py
(load_parameters) against it.
"""
import importlib.util
import json
import os

import yaml

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "codegen_descriptors.json")
KEYS = {  # names of the returned tuple, scripts/<geometry>/common.py return statements
    "diff": ["N", "TF", "DIST_B", "TAU_V", "V_MAX", "A_MAX", "Q_diag", "R_diag", "QN_diag"],
    "omni4": ["N", "TF", "L1_PLUS_L2", "TAU_V", "V_MAX", "A_MAX", "Q_diag", "R_diag", "QN_diag"],
    "tric": ["N", "TF", "DIST_D", "TAU_V", "TAU_A", "V_MAX", "A_MAX", "ALPHA_MIN", "ALPHA_MAX", "DALPHA_MAX",
             "Q_diag", "R_diag", "QN_diag"],
}
VARIATIONS = [{}, {"tf_ini": 1.01, "freq": 20}, {"tf_ini": 1.5, "freq": 30}, {"tf_ini": 0.33, "freq": 50},
              {"tf_ini": 2.0, "freq": 25, "v_max": 0.7, "a_max": 1.5}]


def loader(geometry):
    spec = importlib.util.spec_from_file_location(f"ref_common_{geometry}",
                                                  os.path.join(REF, "scripts", geometry, "common.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.load_parameters


def plain(v):
    if hasattr(v, "tolist"):
        return v.tolist()
    if isinstance(v, (list, tuple)):
        return [plain(x) for x in v]
    return float(v) if not isinstance(v, int) else v


def main():
    shipped = yaml.safe_load(open(os.path.join(REF, "config", "nmpc_nav_control_acados_models.yaml")))
    cases = []
    for geometry in ("diff", "omni4", "tric"):
        load = loader(geometry)
        for var in VARIATIONS + ([{"alpha_min": -20.0, "alpha_max": 35.0, "dalpha_max": 90.0}]
                                 if geometry == "tric" else []):
            params = dict(shipped[f"{geometry}_params"], **var)
            out = load(params)
            cases.append({"geometry": geometry, "params": params,
                          "load_parameters": dict(zip(KEYS[geometry], [plain(v) for v in out]))})
    with open(OUT, "w") as fh:
        json.dump({"source": "scripts/{diff,omni4,tric}/common.py:load_parameters of the reference",
                   "cases": cases}, fh, indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
