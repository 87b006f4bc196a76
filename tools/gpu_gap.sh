set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --cpu-seconds 0 --no-timing > gpurun_out/gap/nt.json 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/gap/t.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o nt -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-timing > gpurun_out/gap/prof.log 2>&1 || exit 1
python3 -c "import json; [print(f, json.loads(open('gpurun_out/gap/'+f).read().strip().splitlines()[-1])['value']) for f in ['nt.json','t.json']]"
