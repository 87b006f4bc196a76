# PMC counter passes (each its own rocprofv3 run, kernel-trace style only) over a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
i=0
for set in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/$TAG -o p$i -- python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-timing --optimize-steps 0 > gpurun_out/$TAG/p$i.log 2>&1 || { tail -20 gpurun_out/$TAG/p$i.log; exit 1; }
done
ls gpurun_out/$TAG
