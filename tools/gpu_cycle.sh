# one build-measure cycle on the GPU box: parity tests, bench, kernel-trace profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cycle}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['kernel_timing_us'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o prof -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-timing > gpurun_out/$TAG/prof.log 2>&1 || { tail -20 gpurun_out/$TAG/prof.log; exit 1; }
cut -d, -f1-4 gpurun_out/$TAG/prof_kernel_stats.csv | head -8
