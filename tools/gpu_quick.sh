# tests + bench of the product library and listed variants + stamps of the stamps library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
bash tools/gpu_profvar.sh base "$@" || exit 1
STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_stamps.so timeout -k 10 300 python tools/stamps.py 512 256 > gpurun_out/$TAG/stamps.log 2>&1 || { tail -20 gpurun_out/$TAG/stamps.log; exit 1; }
head -40 gpurun_out/$TAG/stamps.log
