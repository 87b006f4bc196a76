# cfg3 per-GPU shape with and without pregen
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg3
for envs in STOMP_PREGEN=1 STOMP_PREGEN=0; do
  env $envs timeout -k 10 200 python3 bench.py --waypoints 200 --rollouts-per-gpu 512 --cpu-seconds 0 --optimize-steps 0 --steps 100 --warmup 10 > gpurun_out/cfg3/$envs.json 2> gpurun_out/cfg3/$envs.err || { tail -5 gpurun_out/cfg3/$envs.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfg3/$envs.json')); print('$envs', d['value'], d['kernel_timing_us'])"
done
