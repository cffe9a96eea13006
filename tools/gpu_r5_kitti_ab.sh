# Library A/B on the 1241x376 / 2000-feature mono stream (bench.py --config kitti, B = 256, no extras /
# CPU legs, 40 timed steps after 20 warm-up steps), after the extraction parity tests under each library.
# usage: ROUNDS=3 bash tools/gpu_r5_kitti_ab.sh <tag> lib1 lib2 ...   (names without .so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for lib in "$@"; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par_${lib}.log 2>&1
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 python3 -u bench.py --config kitti --no-cpu-baseline --no-extras --steps 40 --warmup 20 > gpurun_out/${tag}_${lib}_$r.log 2>&1
  done
done
echo KABDONE
