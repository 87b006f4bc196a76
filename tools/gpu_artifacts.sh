# Round artifacts on one box: default bench line (with cpu_baseline), rocprofv3 kernel-trace
# summary of the same workload, PMC traffic passes; outputs under gpurun_out/art
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/art
timeout -k 10 400 python3 bench.py > gpurun_out/art/bench.json 2> gpurun_out/art/bench.err || { tail -20 gpurun_out/art/bench.err; exit 1; }
cat gpurun_out/art/bench.json
bash tools/gpu_prof.sh art_prof || exit 1
bash tools/gpu_pmc.sh art_pmc || exit 1
python3 tools/pmc_traffic.py gpurun_out/art_pmc gpurun_out/art/traffic.json
