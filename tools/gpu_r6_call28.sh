# Round-6 call 28: describe phase stamps (DESC_STAMPS, one slot per wave) of the
# MFMA blur (liborbgpu_xs) and the VALU blur (liborbgpu_xb) at B=512; then the
# grouped kernel at 1 slot per wave (liborbgpu_g1) vs 2 (default) vs the VALU blur.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6ag}
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xs.so timeout -k 10 120 python3 -u tools/extract_stamps.py 512 > gpurun_out/${tag}_stamps_mfma.json 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xb.so timeout -k 10 120 python3 -u tools/extract_stamps.py 512 > gpurun_out/${tag}_stamps_valu.json 2>&1
NO_PMC=1 ROUNDS=2 bash tools/gpu_r6_libab.sh ${tag} liborbgpu_g1 liborbgpu liborbgpu_base
echo CALL28DONE
