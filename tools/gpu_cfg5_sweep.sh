# cfg5 throughput vs problems per GPU (one engine and stream each), optional env as args
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg5
for P in 1 2 4 8; do
  env "$@" timeout -k 10 200 python3 bench.py --problems $P --rollouts-per-gpu 128 --steps 100 --warmup 10 > gpurun_out/cfg5/p$P.json 2> gpurun_out/cfg5/p$P.err || { tail -5 gpurun_out/cfg5/p$P.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfg5/p$P.json')); print('P=$P', d['value'], d['ms_per_step'])"
done
