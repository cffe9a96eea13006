# Round-6 call 14: the whole -m gpu suite on the default build (octree lists of
# <= 64 nodes ordered and pushed by wave 0 alone), then default vs HEAD
# (liborbgpu_base): bench A/B and the single-frame kernel timelines.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6r_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6r_tests.log; exit $rc; }
tail -1 gpurun_out/r6r_tests.log
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh r6r liborbgpu liborbgpu_base
ROUNDS=0 bash tools/gpu_r6_single3.sh r6r_new new:liborbgpu
ROUNDS=0 bash tools/gpu_r6_single3.sh r6r_base base:liborbgpu_base
echo CALL14DONE
