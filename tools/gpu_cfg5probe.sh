set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 200 python3 bench.py --rollouts-per-gpu 128 --cpu-seconds 0 --optimize-steps 0 > gpurun_out/c5/k128.json 2>&1 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c5/k128.json')); print('K128 single', d['value'], d['kernel_timing_us'])"
for P in 2 4 8 16; do
timeout -k 10 200 python3 bench.py --problems $P --rollouts-per-gpu 128 --steps 100 --warmup 10 > gpurun_out/c5/p$P.json 2>&1 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c5/p$P.json')); print('P', $P, d['value'], d['ms_per_step'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/prof -o run -- python3 bench.py --problems 8 --rollouts-per-gpu 128 --steps 50 --warmup 5 > gpurun_out/c5/prof.log 2>&1 || exit 1
head -12 gpurun_out/c5/prof/run_kernel_stats.csv | cut -d, -f1-4
