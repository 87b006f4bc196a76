# The one entry point for GPU-box runs: gpurun -- bash tools/gpu.sh <command> [args].  Every GPU
# step runs under its own time limit and the first failure ends the script; outputs go under
# gpurun_out/ (copy what is to be judged into profiles/).
#
#   tests [FILES]            pytest -m gpu (default: all of tests/), log gpurun_out/t/tests.log
#   smoke                    __graft_entry__.smoke()
#   ab LABEL:ENV[:ARGS] ...  bench.py variants: ENV = VAR=val[,VAR=val] (STOMP_ENGINE_LIB=<path> for
#                            a variant build, STOMP_ROLLOUT=..., any STOMP_DEBUG_*), ARGS = extra
#                            bench arguments with ',' for spaces; each runs 200 steps after 20
#                            warm-ups and the driver's 20 after 5 and prints the per-stage events
#   bench TAG [ARGS]         bench.py ARGS > gpurun_out/TAG.json
#   all TAG                  bench lines of every BASELINE workload (CPU_SECONDS, default 0)
#   prof TAG [ARGS]          rocprofv3 --kernel-trace --stats of bench.py ARGS (default: cfg2, 200
#                            steps after 20) -> gpurun_out/TAG/
#   pmc TAG [ARGS]           the PMC passes (FETCH_SIZE; WRITE_SIZE + TCC hit/miss; SQ counters),
#                            each its own rocprofv3 run, over bench.py ARGS -> gpurun_out/TAG/
#   art R [ARGS]             round artifacts of one workload: prof + pmc + tools/pmc_traffic.py
#                            summary (gpurun_out/art_R/traffic.json) + its bench line (with that
#                            summary and the CPU baselines, ART_CPU seconds, default 12)
#   final R                  tests + smoke + art R for cfg2 + the driver-shape bench line
#   round R                  final R, then art R_cfgX for cfg1 / cfg3 / cfg4 / cfg5 and the
#                            per-rank compute of the sharded shapes (gather 8 4 2, split 64 128 256)
#   stamps LIB K [GRID DOF]  in-kernel phase stamps (tools/stamps.py) with the stamps library LIB
#   micro                    FETCH_SIZE calibration of 2-byte scattered loads (tools/micro/gather_fetch)
#   gather W ...             gather-mode ranks on one GPU (STOMP_DEBUG_GATHER_RANKS=W), cfg2
#   split K ...              the sharded weights phases at per-rank K (STOMP_DEBUG_SHARDED_MODES)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cmd=$1; shift
show() {  # one-line summary of a bench JSON
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], round(d['value'],1), d.get('ms_per_step'), {k: v for k, v in (d.get('kernel_timing_us') or {}).items() if v}, r.get('frac'))" "$1" "$2"
}
bench_to() {  # bench_to OUT LIMIT ARGS...
  local out=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 bench.py "$@" > $out 2> ${out%.json}.err || { tail -20 ${out%.json}.err; return 1; }
}
case "$cmd" in
tests)
  mkdir -p gpurun_out/t
  timeout -k 10 900 python3 -u -m pytest ${@:-tests} -m gpu -x -v --timeout 150 --timeout-method thread --durations=15 > gpurun_out/t/tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/t/tests.log
  exit $rc ;;
smoke)
  mkdir -p gpurun_out/t
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 1; }
  tail -1 gpurun_out/t/smoke.log ;;
ab)
  mkdir -p gpurun_out/ab
  for spec in "$@"; do
    label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
    [ "$args" = "$rest" ] && args=""
    for shape in "200 20" "20 5"; do
      set -- $shape
      out=gpurun_out/ab/$label.$1.json
      env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python3 bench.py --steps $1 --warmup $2 --cpu-seconds 0 --optimize-steps 0 $(echo "$args" | tr ',' ' ') > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
      show $out "$label $1/$2"
    done
  done ;;
bench)
  tag=$1; shift
  bench_to gpurun_out/$tag.json 600 "$@" || exit 1
  cat gpurun_out/$tag.json ;;
all)
  tag=${1:-all}; cpu=${CPU_SECONDS:-0}
  mkdir -p gpurun_out/$tag
  bench_to gpurun_out/$tag/cfg2.json 400 --cpu-seconds $cpu || exit 1
  bench_to gpurun_out/$tag/cfg2_driver.json 300 --steps 20 --warmup 5 --cpu-seconds 0 --optimize-steps 0 || exit 1
  for w in cfg1 cfg3 cfg4 cfg5; do
    bench_to gpurun_out/$tag/$w.json 400 --workload $w --steps 100 --warmup 10 --cpu-seconds 0 --optimize-steps 0 || exit 1
  done
  for f in gpurun_out/$tag/*.json; do show $f $(basename $f .json); done ;;
prof)
  tag=$1; shift
  mkdir -p gpurun_out/$tag
  [ $# -eq 0 ] && set -- --steps 200 --warmup 20
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 bench.py --cpu-seconds 0 --optimize-steps 0 "$@" > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { tail -30 gpurun_out/$tag/bench.err; exit 1; }
  find gpurun_out/$tag -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20 ;;
pmc)
  tag=$1; shift
  mkdir -p gpurun_out/$tag
  [ $# -eq 0 ] && set -- --steps 40 --warmup 5
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/$tag -o p$i -- python3 bench.py --cpu-seconds 0 --no-timing --optimize-steps 0 "$@" > gpurun_out/$tag/p$i.log 2>&1 || { tail -20 gpurun_out/$tag/p$i.log; exit 1; }
  done
  ls gpurun_out/$tag ;;
art)
  r=$1; shift
  bash tools/gpu.sh prof art_${r}_prof "$@" || exit 1
  bash tools/gpu.sh pmc art_${r}_pmc "$@" || exit 1
  mkdir -p gpurun_out/art_$r
  cp "$(find gpurun_out/art_${r}_prof -name '*kernel_stats.csv' | head -1)" gpurun_out/art_$r/kernel_stats.csv
  wl=cfg2; prev=""
  for a in "$@"; do [ "$prev" = "--workload" ] && wl=$a; prev=$a; done
  python3 tools/pmc_traffic.py gpurun_out/art_${r}_pmc gpurun_out/art_$r/traffic.json gpurun_out/art_$r/kernel_stats.csv $wl || exit 1
  # the bench line reads the PMC summary of its own build from profiles/ (bench.py pmc_summary):
  # this box's copy, so the line carries traffic and VALU (commit traffic.json under profiles/)
  cp gpurun_out/art_$r/traffic.json profiles/_box_${r}_rollout_cost_traffic.json
  bench_to gpurun_out/art_$r/bench.json 500 --cpu-seconds ${ART_CPU:-12} "$@" || exit 1
  cat gpurun_out/art_$r/bench.json ;;
final)
  r=$1
  bash tools/gpu.sh tests || exit 1
  bash tools/gpu.sh smoke || exit 1
  bash tools/gpu.sh art $r || exit 1
  bench_to gpurun_out/art_$r/bench_driver.json 500 --steps 20 --warmup 5 || exit 1
  cat gpurun_out/art_$r/bench_driver.json ;;
round)
  r=$1
  bash tools/gpu.sh final $r || exit 1
  bash tools/gpu.sh art ${r}_cfg1 --workload cfg1 --steps 200 --warmup 20 || exit 1
  bash tools/gpu.sh art ${r}_cfg4 --workload cfg4 --steps 60 --warmup 10 || exit 1
  bash tools/gpu.sh art ${r}_cfg3 --workload cfg3 --steps 20 --warmup 5 || exit 1
  bash tools/gpu.sh art ${r}_cfg5 --workload cfg5 --steps 20 --warmup 5 || exit 1
  bash tools/gpu.sh gather 8 4 2 || exit 1
  bash tools/gpu.sh split 64 128 256 || exit 1 ;;
stamps)
  lib=$1; k=$2; shift 2
  mkdir -p gpurun_out/stamps
  out=gpurun_out/stamps/$(basename $lib .so).$k.txt
  STOMP_ENGINE_LIB=$PWD/$lib timeout -k 10 120 python3 tools/stamps.py $k "$@" > $out 2>&1 || { tail -5 $out; exit 1; }
  head -40 $out ;;
micro)
  # FETCH_SIZE per line for 2-byte scattered loads (tools/micro/gather_fetch.hip, built on the CPU)
  d=gpurun_out/micro; mkdir -p $d
  i=0
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $d/p$i -o p$i -- tools/micro/gather_fetch $d/known.json > $d/p$i.log 2>&1 || { tail -20 $d/p$i.log; exit 1; }
  done
  python3 tools/micro/gather_fetch.py $d $d/gather_fetch.json ;;
gather)
  mkdir -p gpurun_out/split
  for w in "$@"; do
    out=gpurun_out/split/g$w.json
    STOMP_DEBUG_GATHER_RANKS=$w bench_to $out 300 --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 || exit 1
    show $out "gather W=$w K=512"
  done ;;
split)
  mkdir -p gpurun_out/split
  for k in "$@"; do
    for m in 0 1; do
      out=gpurun_out/split/m$m.$k.json
      STOMP_DEBUG_SHARDED_MODES=$m bench_to $out 300 --steps 200 --warmup 20 --cpu-seconds 0 --optimize-steps 0 --rollouts $k || exit 1
      show $out "modes=$m K=$k"
    done
  done ;;
*)
  echo "unknown command $cmd"; exit 2 ;;
esac
