# Round profiles: GPU tests, smoke, PMC traffic passes, the bench line, rocprofv3 kernel stats
# (arg: tag, e.g. r1).  Everything lands under gpurun_out/prof_<tag>/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_pmc.sh prof_$TAG/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc $OUT/${TAG}_rollout_cost_traffic.json || exit 1
cp $OUT/${TAG}_rollout_cost_traffic.json profiles/
timeout -k 10 400 python3 bench.py > $OUT/${TAG}_bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
find $OUT/stats -name "*kernel_stats*"
