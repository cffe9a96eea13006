# Round-6 call 34: CheckInliers over runs of up to 4 consecutive same-candidate
# hypotheses per wave (default) vs up to 3 in groups of 2 (liborbgpu_c2) vs
# pairs (liborbgpu_prev, HEAD); loop / RANSAC GPU tests, loopburst bench x2.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6am}
timeout -k 10 600 python -u -m pytest tests/test_loop.py tests/test_ransac.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/${tag}_tests.log | head -20; exit $rc; }
for r in 1 2; do
  for lib in liborbgpu liborbgpu_c2 liborbgpu_prev; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 300 python3 -u bench.py --config loopburst --no-cpu-baseline > gpurun_out/${tag}_${lib}_$r.log 2>&1 || { echo "$lib failed"; exit 3; }
  done
done
echo CALL34DONE
