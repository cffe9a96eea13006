# Round-6 call 15: the whole -m gpu suite on the default build (octree roots by wave 0,
# the last pass fused with the best-key sweep), then default vs HEAD
# (liborbgpu_base): bench A/B and the single-frame kernel timelines.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6s_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6s_tests.log; exit $rc; }
tail -1 gpurun_out/r6s_tests.log
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh r6s liborbgpu liborbgpu_base
ROUNDS=0 bash tools/gpu_r6_single3.sh r6s_new new:liborbgpu
ROUNDS=0 bash tools/gpu_r6_single3.sh r6s_base base:liborbgpu_base
echo CALL15DONE
