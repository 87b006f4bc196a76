# A/B of the update kernel: GPU tests, the 200-step and driver-shape bench lines, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-upd}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 300 python3 bench.py --cpu-seconds 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/$TAG/bench_driver.json 2> gpurun_out/$TAG/bench_driver.err || { tail -20 gpurun_out/$TAG/bench_driver.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/$TAG/prof.log 2>&1 || { tail -20 gpurun_out/$TAG/prof.log; exit 1; }
for f in gpurun_out/$TAG/bench.json gpurun_out/$TAG/bench_driver.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['kernel_timing_us'])" $f; done
find gpurun_out/$TAG/prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -6
