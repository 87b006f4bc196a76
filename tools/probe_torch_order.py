"""Probe: does the engine library work when torch initialised its bundled HIP runtime first?"""
import sys
order = sys.argv[1]
if order == "torch_first":
    import torch
    torch.cuda.init()
    print("torch devices", torch.cuda.device_count())
from stomp_motion_planner_icra2011_amd import engine as eng, problem as pb
import numpy as np
p = pb.make_problem(grid_n=32, num_rollouts=8, num_reused_rollouts=0)
e = eng.Engine(p)
print(order, "iterate", e.iterate(1))
if order == "engine_first":
    import torch
    try:
        torch.cuda.init(); print("torch ok after engine", torch.cuda.device_count())
    except Exception as ex:
        print("torch failed after engine:", ex)
