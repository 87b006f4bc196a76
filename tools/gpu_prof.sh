# rocprofv3 kernel-trace summary of the default bench workload (run through gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20
