#!/usr/bin/env python3
"""Extracts the constants the reference holds for the hot path into a committed fixture,
tests/golden/reference_constants.json (data only: numbers and the file:line they come from).

Run in the container, where /root/reference exists (the GPU box has no copy):
    python tools/extract_reference_constants.py
Sources (relative to /root/reference/stomp_motion_planner/):
  include/stomp_motion_planner/stomp_utils.h   DIFF_RULES (the 7-tap vel / acc / jerk stencils)
  config/params.yaml                           the loop / optimizer parameters
  src/stomp_parameters.cpp                     StompParameters defaults (node_handle.param)
  config/pr2_both_arms_stomp_config.yaml       collision clearance, sphere radii / extensions, joint costs
  config/environment_shelf.yaml                the 10-box shelf scene
  config/environment_pole.yaml                 the pole
tests/test_reference_constants.py checks the engine, the oracle and problem.py against it.
"""
import json
import os
import re
import sys

import yaml

REF = os.environ.get("STOMP_REFERENCE", "/root/reference/stomp_motion_planner")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "reference_constants.json")


def lines_of(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read().split("\n")


def c_double(expr: str) -> float:
    """A C constant expression of the DIFF_RULES table: an int or double literal, optionally
    divided by a double literal (the int converts to double, then one IEEE division)."""
    expr = expr.strip()
    m = re.fullmatch(r"(-?\d+(?:\.\d*)?)\s*/\s*(\d+\.\d*)", expr)
    if m:
        return float(m.group(1)) / float(m.group(2))
    return float(expr)


def diff_rules():
    rel = "include/stomp_motion_planner/stomp_utils.h"
    L = lines_of(rel)
    start = next(i for i, l in enumerate(L) if "DIFF_RULES[NUM_DIFF_RULES][DIFF_RULE_LENGTH]" in l)
    rows, i = [], start + 1
    while len(rows) < 3:
        m = re.search(r"\{([^}]*)\}", L[i])
        if m:
            rows.append([c_double(x) for x in m.group(1).split(",")])
        i += 1
    return {"value": rows, "source": f"{rel}:{start + 1}-{i}"}


def yaml_file(rel):
    with open(os.path.join(REF, rel)) as f:
        return yaml.safe_load(f), f"{rel}:1-{len(lines_of(rel))}"


def parameter_defaults():
    rel = "src/stomp_parameters.cpp"
    out = {}
    for n, l in enumerate(lines_of(rel), 1):
        m = re.search(r'node_handle\.param\("(\w+)",\s*\w+,\s*([^)]+)\)', l)
        if m:
            v = m.group(2).strip()
            if v in ("true", "false"):
                val = v == "true"
            else:
                try:
                    val = float(v)
                except ValueError:
                    continue   # string-valued parameters (frames, names) are off the path
            out[m.group(1)] = {"value": val, "source": f"{rel}:{n}"}
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit(f"reference not found at {REF}")
    params, params_src = yaml_file("config/params.yaml")
    stomp_cfg, stomp_src = yaml_file("config/pr2_both_arms_stomp_config.yaml")
    shelf, shelf_src = yaml_file("config/environment_shelf.yaml")
    pole, pole_src = yaml_file("config/environment_pole.yaml")
    fixture = {
        "note": "constants held by kalakris/stomp_motion_planner_icra2011 (data extracted by "
                "tools/extract_reference_constants.py; paths relative to stomp_motion_planner/)",
        "diff_rules": diff_rules(),
        "params": {"value": params, "source": params_src},
        "parameter_defaults": parameter_defaults(),
        "stomp_config": {"value": {"collision_clearance": stomp_cfg["collision_clearance"],
                                   "collision_links": stomp_cfg["collision_links"],
                                   "joint_costs": stomp_cfg.get("joint_costs", {})},
                         "source": stomp_src},
        "shelf_boxes": {"value": shelf["boxes"], "source": shelf_src},
        "pole_cylinders": {"value": pole["cylinders"], "source": pole_src},
    }
    with open(OUT, "w") as f:
        json.dump(fixture, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
