# phase stamps of the product and a variant kernel: args "variant:K"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/stamps
for vk in "$@"; do
  v=${vk%%:*}; k=${vk##*:}
  STOMP_ENGINE_LIB=$PWD/stomp_motion_planner_icra2011_amd/libstomp_engine_$v.so timeout -k 10 120 python3 tools/stamps.py $k > gpurun_out/stamps/$v.$k.txt 2>&1 || { tail -5 gpurun_out/stamps/$v.$k.txt; exit 1; }
done
