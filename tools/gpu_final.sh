# Round-end evidence at this build: GPU tests + smoke, then tools/gpu_artifacts.sh (kernel stats,
# PMC traffic of this build, driver-shape and 200-step bench lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r3}
mkdir -p gpurun_out/art
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/art/gpu_tests.log 2>&1 || { tail -30 gpurun_out/art/gpu_tests.log; exit 1; }
tail -1 gpurun_out/art/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/art/smoke.log 2>&1 || { tail -20 gpurun_out/art/smoke.log; exit 1; }
tail -1 gpurun_out/art/smoke.log
bash tools/gpu_artifacts.sh $R
