set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export ORBGPU_PYR_MODE=band
for v in stamps stampsetup; do
  ORBGPU_LIBRARY=$PWD/exp/$v/liborbgpu.so timeout -k 10 120 python tools/pyr_stamps.py > gpurun_out/st_$v.log 2>&1 || true
done
