# Round artifacts on one box (run through gpurun): rocprofv3 kernel-trace summary of the default
# bench workload, the PMC passes (tools/gpu_pmc.sh) and their per-launch summary with the VALU
# issue fraction, then the default bench line (driver shape and 200 steps), which reads that
# summary because it is of this very build.  Outputs under gpurun_out/art; copy
# gpurun_out/art/{kernel_stats.csv,traffic.json,bench*.json} into profiles/<round>_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r3}
mkdir -p gpurun_out/art
bash tools/gpu_prof.sh art_prof || exit 1
cp "$(find gpurun_out/art_prof -name '*kernel_stats.csv' | head -1)" gpurun_out/art/kernel_stats.csv
bash tools/gpu_pmc.sh art_pmc || exit 1
python3 tools/pmc_traffic.py gpurun_out/art_pmc gpurun_out/art/traffic.json gpurun_out/art/kernel_stats.csv || exit 1
cp gpurun_out/art/traffic.json profiles/${R}_rollout_cost_traffic.json
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/art/bench_driver.json 2> gpurun_out/art/bench_driver.err || { tail -20 gpurun_out/art/bench_driver.err; exit 1; }
cat gpurun_out/art/bench_driver.json
timeout -k 10 400 python3 bench.py --cpu-seconds 0 > gpurun_out/art/bench.json 2> gpurun_out/art/bench.err || { tail -20 gpurun_out/art/bench.err; exit 1; }
cat gpurun_out/art/bench.json
