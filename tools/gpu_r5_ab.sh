# Round-5 A/B call: parity (+ extra test files given), then the bench line
# (no extras / CPU legs, 40 timed steps after 20 warm-up steps) under each
# value of $AB_VAR listed in $AB_VALS, interleaved over $ROUNDS rounds, then
# the same for each library in $AB_LIBS (names without .so).
# usage: AB_VAR=ORBGPU_FAST_DMA AB_VALS="0 4" AB_LIBS="liborbgpu_x" bash tools/gpu_r5_ab.sh <tag> [test files...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py "$@" > gpurun_out/${tag}_par.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${AB_VALS}; do
    env ${AB_VAR}=$v timeout -k 10 200 $B > gpurun_out/${tag}_${AB_VAR}${v}_$r.log 2>&1 || echo "$v failed"
  done
  for lib in ${AB_LIBS}; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 $B > gpurun_out/${tag}_${lib}_$r.log 2>&1 || echo "$lib failed"
  done
done
echo ABDONE
