set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['kernel_timing_us'], d['roofline'])"
STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_stamps.so timeout -k 10 300 python tools/stamps.py 512 256 > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
