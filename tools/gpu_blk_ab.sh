set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/blk
for v in b512 b1024; do
  STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/blk/tests_$v.log 2>&1 || { tail -20 gpurun_out/blk/tests_$v.log; exit 1; }
  tail -1 gpurun_out/blk/tests_$v.log
done
bash tools/gpu_ab.sh base:64 b512:64 b1024:64 base:128 b512:128 b1024:128 base:256 b512:256 base:512 b512:512
