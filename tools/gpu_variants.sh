# timing of experiment library variants (bench kernel timings), run through gpurun
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for v in "$@"; do
  lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine${v:+_$v}.so
  [ "$v" = "base" ] && lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine.so
  STOMP_ENGINE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { tail -5 gpurun_out/var/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var/$v.json')); print('$v', d['value'], d['kernel_timing_us'])"
done
