# Octree check: extractor parity, phase stamps (diagnostic build), bench line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-oct}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_os.so timeout -k 10 120 python3 tools/octree_trace.py 512 > gpurun_out/${tag}_stamps.txt 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo OCTDONE
