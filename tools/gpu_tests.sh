# GPU test suite (all -m gpu tests, or the files given as arguments), one process, logs under gpurun_out/t/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t
files="${@:-tests}"
timeout -k 10 900 python3 -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/t/tests.log 2>&1
rc=$?
tail -30 gpurun_out/t/tests.log
exit $rc
