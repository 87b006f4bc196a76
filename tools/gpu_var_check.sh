# parity of a library variant (test_gpu_parity + test_gpu_configs), then A/B lines: args variant "variant:K" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
v=$1; shift
STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
tail -1 gpurun_out/var_$v.log
bash tools/gpu_ab.sh "$@"
