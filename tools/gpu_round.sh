# GPU tests of the product library, then the round artifacts (bench line, rocprof stats, PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t/tests.log 2>&1 || { tail -40 gpurun_out/t/tests.log; exit 1; }
tail -3 gpurun_out/t/tests.log
bash tools/gpu_artifacts.sh
