# rocprof kernel stats for a list of library variants (base = product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so
  [ "$v" = "base" ] && lib=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine.so
  mkdir -p gpurun_out/pv_$v
  STOMP_ENGINE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv_$v -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-timing > gpurun_out/pv_$v/bench.json 2> gpurun_out/pv_$v/err.log || { tail -5 gpurun_out/pv_$v/err.log; exit 1; }
  echo "=== $v $(python3 -c "import json; print(json.load(open('gpurun_out/pv_$v/bench.json'))['value'])")"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/pv_$v/run_kernel_stats.csv')):
    if 'stomp::' in r['Name']: print('  %-45s %6s %9.2f us' % (r['Name'].split('(')[0][-45:], r['Calls'], float(r['AverageNs']) / 1000))
"
done
