# SQ counter passes for the rollout kernel (each its own rocprofv3 run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmcsq}
mkdir -p gpurun_out/$TAG
timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/$TAG -o q$i -- python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-timing > gpurun_out/$TAG/q$i.log 2>&1 || { tail -20 gpurun_out/$TAG/q$i.log; exit 1; }
done
ls gpurun_out/$TAG
