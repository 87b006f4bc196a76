# does the short driver-shaped run (20 steps after 5 warm-ups) lose to clock ramp or to iteration
# content?  bench variants + a kernel trace of the long run (per-dispatch k_rollout durations)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/warm
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 200" "--steps 200 --warmup 5" "--steps 20 --warmup 5"; do
  timeout -k 10 120 python3 bench.py $args --cpu-seconds 0 --optimize-steps 0 > gpurun_out/warm/b.json 2>gpurun_out/warm/b.err || { tail gpurun_out/warm/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/warm/b.json')); print('$args', d['value'], d['kernel_timing_us'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/warm/kt -o kt -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 --no-timing > gpurun_out/warm/kt.log 2>&1 || { tail gpurun_out/warm/kt.log; exit 1; }
find gpurun_out/warm/kt -name "*kernel_trace.csv" | head
