# GPU tests, then bench lines with and without the side-stream pregen (args: extra env settings to A/B, e.g. STOMP_PREGEN=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/chk
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk/tests.log 2>&1 || { tail -40 gpurun_out/chk/tests.log; exit 1; }
tail -2 gpurun_out/chk/tests.log
i=0
for envs in "" "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/chk/b$i.json 2> gpurun_out/chk/b$i.err || { tail -5 gpurun_out/chk/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/chk/b$i.json')); print('[$envs]', d['value'], d['kernel_timing_us'], d.get('optimize_loop'))"
done
