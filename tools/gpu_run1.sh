set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests_2.log 2>&1 || { tail -30 gpurun_out/gpu_tests_2.log; exit 1; }
tail -3 gpurun_out/gpu_tests_2.log
timeout -k 10 120 python tools/probe_torch_order.py torch_first > gpurun_out/probe1.log 2>&1; echo "probe1 rc=$?"; tail -3 gpurun_out/probe1.log
timeout -k 10 120 python tools/probe_torch_order.py engine_first > gpurun_out/probe2.log 2>&1; echo "probe2 rc=$?"; tail -3 gpurun_out/probe2.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-timing > gpurun_out/prof1.log 2>&1 || { tail -20 gpurun_out/prof1.log; exit 1; }
find gpurun_out/prof1 -name "*stats*" | head
