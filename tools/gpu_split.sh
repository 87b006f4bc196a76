# split pipeline vs fused k_rollout: bench lines (long and driver-shaped), env A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/split
for env in "STOMP_SPLIT=1" "STOMP_SPLIT=0"; do
  for args in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    env $env timeout -k 10 200 python3 bench.py $args --cpu-seconds 0 --optimize-steps 0 > gpurun_out/split/b.json 2> gpurun_out/split/b.err || { tail -5 gpurun_out/split/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/split/b.json')); print('$env $args', d['value'], d['kernel_timing_us'])"
  done
done
