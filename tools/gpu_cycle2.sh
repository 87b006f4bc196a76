# tests + bench of the product library + timings of listed variants + stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cyc}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
for v in base "$@"; do
  lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so
  [ "$v" = "base" ] && lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine.so
  STOMP_ENGINE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err || { tail -5 gpurun_out/$TAG/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/$v.json')); print('$v', d['value'], d['kernel_timing_us'])"
done
STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_stamps.so timeout -k 10 300 python tools/stamps.py 512 256 > gpurun_out/$TAG/stamps.log 2>&1 || { tail -20 gpurun_out/$TAG/stamps.log; exit 1; }
cat gpurun_out/$TAG/stamps.log
