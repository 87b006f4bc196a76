# the sharded weights phases (W_MINMAX / W_PSUM / W_USUM with one-rank identity exchanges) on
# one GPU at per-rank shard sizes: the compute side of a K-sharded iteration
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
for k in "$@"; do
  for m in 0 1; do
    STOMP_DEBUG_SHARDED_MODES=$m timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 --rollouts $k > gpurun_out/split/m$m.$k.json 2> gpurun_out/split/m$m.$k.err || { tail -5 gpurun_out/split/m$m.$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/split/m$m.$k.json')); print('modes=$m K=$k', d['value'], d['ms_per_step'], d['kernel_timing_us'])"
  done
done
