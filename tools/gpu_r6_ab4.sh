# Round-6 call 4: the whole -m gpu suite on the default build (FAST ring pairs by
# ds_read_u8_d16/_hi, batch octree with wave-aggregated quadrant counts), then
# the default against the build without the d16 ring reads.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6e}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_nod16
echo AB4DONE
