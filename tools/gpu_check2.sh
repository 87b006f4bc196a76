# one engine creation with the phased-layout report, the full GPU suite, A/B lines, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STOMP_DEBUG_PHASED=1 timeout -k 10 120 python3 -c "
from stomp_motion_planner_icra2011_amd import engine as eng, problem as pb
p = pb.make_problem(dof=7, waypoints=100, grid_n=64, num_rollouts=64, num_reused_rollouts=0)
e = eng.Engine(p); e.run(1, 3); e.synchronize(); print('ok')
" 2>&1 | tail -3 || exit 1
bash tools/gpu_check.sh "$@" || exit 1
bash tools/gpu_stamps.sh stamps:64
