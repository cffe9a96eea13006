# Round-6 call 17: octree phase stamps at B=1 and B=512 (OCT_STAMPS build) after
# the wave-0 small-list passes.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_os.so timeout -k 10 120 python3 -u tools/octree_trace.py 1 > gpurun_out/r6u_oct1.txt 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_os.so timeout -k 10 120 python3 -u tools/octree_trace.py 512 > gpurun_out/r6u_oct512.txt 2>&1
echo CALL17DONE
