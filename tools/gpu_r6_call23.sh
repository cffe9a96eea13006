# Round-6 call 23: MFMA blur variants -- tap fragments loaded at the kernel's
# start (default) vs just before the blur (liborbgpu_mf1) vs the VALU blur
# (liborbgpu_base); bench A/B only.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6ab}
NO_PMC=1 ROUNDS=2 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_mf1 liborbgpu_base
echo CALL23DONE
