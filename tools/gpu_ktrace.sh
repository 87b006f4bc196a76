# rocprofv3 kernel trace + stats of a short bench (env passed through), summary per kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-kt}
mkdir -p gpurun_out/$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o kt -- python3 bench.py --steps 50 --warmup 10 --cpu-seconds 0 --optimize-steps 0 --no-timing > gpurun_out/$TAG/kt.log 2>&1 || { tail -20 gpurun_out/$TAG/kt.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/$TAG/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], r["AverageNs"], r["Percentage"])
PY
