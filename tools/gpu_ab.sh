# GPU tests, then bench A/B of an env switch (default vs "$1"=1); outputs under gpurun_out/ab
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -40 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
for v in 0 1; do
  env $1=$v timeout -k 10 200 python3 bench.py --cpu-seconds 0 > gpurun_out/ab/b$v.json 2> gpurun_out/ab/b$v.err || { tail -20 gpurun_out/ab/b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/b$v.json')); print('$1=$v', d['value'], d['kernel_timing_us'], d['optimize_loop'])"
done
