# cfg3's per-rank shard at 8 GPUs (K_loc = 512, N = 199) and the whole K on one GPU: the compute
# side of the K split (modes=1: the sharded weights phases with one-rank identity exchanges)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
for m in 0 1; do
  STOMP_DEBUG_SHARDED_MODES=$m timeout -k 10 200 python3 bench.py --workload cfg3 --rollouts 512 --steps 100 --warmup 10 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/split/cfg3_m$m.512.json 2> gpurun_out/split/cfg3_m$m.512.err || { tail -5 gpurun_out/split/cfg3_m$m.512.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/split/cfg3_m$m.512.json')); print('cfg3 modes=$m K=512', d['value'], d['ms_per_step'], d['kernel_timing_us'])"
done
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 30 --warmup 5 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/split/cfg3_whole.json 2> gpurun_out/split/cfg3_whole.err || { tail -5 gpurun_out/split/cfg3_whole.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/split/cfg3_whole.json')); print('cfg3 whole K=4096', d['value'], d['ms_per_step'], d['kernel_timing_us'])"
