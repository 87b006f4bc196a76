# A/B of one library under environment settings: args "name:VAR=value" ("name:" = no setting)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { tail -5 gpurun_out/ab/$name.err; exit 1; }
  env $envs timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/ab/$name.short.json 2> gpurun_out/ab/$name.short.err || { tail -5 gpurun_out/ab/$name.short.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$name.json')); s=json.load(open('gpurun_out/ab/$name.short.json')); print('$name', d['value'], d['kernel_timing_us']['rollout_cost'], 'short', s['value'], s['kernel_timing_us']['rollout_cost'])"
done
