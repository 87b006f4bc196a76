# stamps + residency diagnostics for one or more stamps-enabled library variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/st
for v in "${@:-stamps}"; do
  echo "=== $v"
  STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so timeout -k 10 300 python tools/stamps.py 512 256 > gpurun_out/st/$v.log 2>&1 || { tail -20 gpurun_out/st/$v.log; exit 1; }
  cat gpurun_out/st/$v.log
done
