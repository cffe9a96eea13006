# Round-5 iteration call: the GPU tests given (default: extraction parity and
# the adapter tests), the bench line (no extras / CPU legs, 40 timed steps
# after 20 warm-up steps) for each library named, interleaved over $ROUNDS
# rounds, then the stereo drop-in tail (tools/gpu_r5_stereo.sh) when STEREO=1.
# usage: ROUNDS=2 bash tools/gpu_r5_iter.sh <tag> lib1 [lib2 ...]   (names without .so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_adapter.py} > gpurun_out/${tag}_par.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20 > gpurun_out/${tag}_${lib}_$r.log 2>&1
  done
done
if [ "${STEREO:-0}" = 1 ]; then REPS=1000 bash tools/gpu_r5_stereo.sh ${tag}; fi
echo ITERDONE
