# gather-mode ranks timed on one GPU (STOMP_DEBUG_GATHER_RANKS=W: rank 0 of W, its K / W rollouts
# evaluated, all K noise rows made and priced, weights over all K, nothing exchanged), next to
# the whole K on one device; args: W values (cfg2, K = 512)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
for w in "$@"; do
  STOMP_DEBUG_GATHER_RANKS=$w timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/split/g$w.json 2> gpurun_out/split/g$w.err || { tail -5 gpurun_out/split/g$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/split/g$w.json')); print('gather W=$w K=512', d['value'], d['ms_per_step'], d['kernel_timing_us'])"
done
