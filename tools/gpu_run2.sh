set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-timing > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')):
    print(f"{r['Name'][:50]:50s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1000:9.2f} pct={float(r['Percentage']):6.2f}")
PY
