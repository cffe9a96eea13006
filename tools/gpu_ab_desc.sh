set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/q5_gpu.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/q5_bench4.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_d8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/q5_gpu8.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_d8.so timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/q5_bench8.log 2>&1
echo CMPDONE
