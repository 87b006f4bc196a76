# GPU tests (incl. the one-rank RCCL path), cfg1 timings, default bench line; outputs under gpurun_out/r1b
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r1b
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u tools/cfg1.py --iterations 500 > $OUT/cfg1.json 2> $OUT/cfg1.err || { tail -20 $OUT/cfg1.err; exit 1; }
cat $OUT/cfg1.json
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
