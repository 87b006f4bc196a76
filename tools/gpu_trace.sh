# kernel timeline of a short bench run (rocprofv3 kernel trace), env settings as args
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/trace
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/trace/t$i -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 --no-timing --optimize-steps 0 > gpurun_out/trace/t$i.log 2>&1 || { tail -20 gpurun_out/trace/t$i.log; exit 1; }
done
find gpurun_out/trace -name "*kernel_trace*"
