# Round-6 A/B call 1: FAST XCD-local cell runs (sw2), describe LDS-conflict
# probes (dp*), single-frame octree thread counts (o256/o512).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUNDS=2 bash tools/gpu_r6_libab.sh r6b liborbgpu liborbgpu_sw2 liborbgpu_dp1 liborbgpu_dp2 liborbgpu_dp4 liborbgpu_dp8 liborbgpu_dp15
ROUNDS=3 bash tools/gpu_r6_single.sh r6b liborbgpu liborbgpu_o256 liborbgpu_o512
echo AB1DONE
