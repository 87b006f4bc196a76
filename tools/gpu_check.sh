# full GPU test suite, then A/B lines of the product library at the given rollout counts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
[ $# -gt 0 ] && bash tools/gpu_ab.sh "$@"
exit 0
