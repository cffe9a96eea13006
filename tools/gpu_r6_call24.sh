# Round-6 call 24: latency probe -- describe with every keypoint's neighbourhood
# read from frame 0's level 0 (DESC_PROBE_SAMEFRAME: L2-resident, wrong results)
# for the MFMA blur (liborbgpu_pm) and the VALU blur (liborbgpu_pb).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6ac}
NO_PMC=1 ROUNDS=2 bash tools/gpu_r6_libab.sh ${tag} liborbgpu_pm liborbgpu_pb
echo CALL24DONE
