# bench lines for every BASELINE workload on one GPU (outputs under gpurun_out/<tag>/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-bench}
CPU=${CPU_SECONDS:-12}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 bench.py --cpu-seconds $CPU > gpurun_out/$TAG/cfg2.json 2> gpurun_out/$TAG/cfg2.err || { tail -20 gpurun_out/$TAG/cfg2.err; exit 1; }
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/$TAG/cfg2_driver.json 2> gpurun_out/$TAG/cfg2_driver.err || { tail -20 gpurun_out/$TAG/cfg2_driver.err; exit 1; }
for w in cfg1 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 100 --warmup 10 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/$TAG/$w.json 2> gpurun_out/$TAG/$w.err || { tail -20 gpurun_out/$TAG/$w.err; exit 1; }
done
for f in gpurun_out/$TAG/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d.get('kernel_timing_us'), (d.get('roofline') or {}).get('frac'))"; done
