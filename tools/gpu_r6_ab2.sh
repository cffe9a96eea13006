# Round-6 call 2: extraction parity with the default build, FAST / describe phase
# stamps at B=512 (FAST_STAMPS/DESC_STAMPS build), octree phase stamps at B=1 and
# B=512 (OCT_STAMPS build).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6c}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_parity.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xs.so timeout -k 10 120 python3 -u tools/extract_stamps.py 512 > gpurun_out/${tag}_stamps512.json 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xs.so timeout -k 10 120 python3 -u tools/extract_stamps.py 1 > gpurun_out/${tag}_stamps1.json 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_os.so timeout -k 10 120 python3 -u tools/octree_trace.py 1 > gpurun_out/${tag}_oct1.txt 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_os.so timeout -k 10 120 python3 -u tools/octree_trace.py 512 > gpurun_out/${tag}_oct512.txt 2>&1
echo AB2DONE
