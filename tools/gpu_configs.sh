# Bench lines for the BASELINE configs on one GPU (cfg2 default, cfg3 per-GPU shard shape,
# cfg4 dual-arm 512^3, cfg5 8 problems per GPU); outputs under gpurun_out/cfg
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
run() {
  name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > gpurun_out/cfg/$name.json 2> gpurun_out/cfg/$name.err || { tail -20 gpurun_out/cfg/$name.err; exit 1; }
  cat gpurun_out/cfg/$name.json
}
run cfg2 --cpu-seconds 0
run cfg3_shard --waypoints 200 --rollouts-per-gpu 512 --cpu-seconds 0 --optimize-steps 0
run cfg4 --dof 14 --rollouts-per-gpu 1024 --grid 512 --cpu-seconds 0 --optimize-steps 0
run cfg5 --problems 8 --rollouts-per-gpu 128 --steps 100 --warmup 10
