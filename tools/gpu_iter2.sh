set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ORBGPU_LIBRARY=$PWD/exp/stamps/liborbgpu.so timeout -k 10 120 python tools/pyr_stamps.py > gpurun_out/stamps.log 2>&1
rm -rf exp/stamps
bash tools/variants_kstats.sh
