# A/B of library variants at given rollout counts: args "variant:K" (variant "base" = product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for vk in "$@"; do
  v=${vk%%:*}; k=${vk##*:}
  lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so
  [ "$v" = "base" ] && lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine.so
  STOMP_ENGINE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --rollouts $k --optimize-steps 0 > gpurun_out/ab/$v.$k.json 2> gpurun_out/ab/$v.$k.err || { tail -5 gpurun_out/ab/$v.$k.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.$k.json')); print('$v K=$k', d['value'], d['kernel_timing_us'])"
done
# the driver's shape: 20 steps after 5 warm-ups (the heavier early iterations)
for vk in "$@"; do
  v=${vk%%:*}; k=${vk##*:}
  lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so
  [ "$v" = "base" ] && lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine.so
  STOMP_ENGINE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --rollouts $k --optimize-steps 0 > gpurun_out/ab/$v.$k.short.json 2> gpurun_out/ab/$v.$k.short.err || { tail -5 gpurun_out/ab/$v.$k.short.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.$k.short.json')); print('$v K=$k short', d['value'], d['kernel_timing_us']['rollout_cost'])"
done
