set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_stamps.so timeout -k 10 300 python tools/stamps.py 512 256 > gpurun_out/stamps.log 2>&1; rc=$?
cat gpurun_out/stamps.log | tail -80
exit $rc
