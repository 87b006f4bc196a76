# WG-count probe for the given library variants ("base" = product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
for v in "$@"; do
  lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so
  [ "$v" = "base" ] && lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine.so
  STOMP_ENGINE_LIB=$lib timeout -k 10 200 python3 tools/wg_count_probe.py 6 > gpurun_out/probe/$v.txt 2>&1 || { tail -5 gpurun_out/probe/$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/probe/$v.txt
done
