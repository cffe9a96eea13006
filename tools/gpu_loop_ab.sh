# Loop burst A/B (compute_sim3 block size): loop parity, then the loopburst bench per library.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_loop.py tests/test_ransac.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lp_gpu.log 2>&1
timeout -k 10 300 python3 -u bench.py --config loopburst --no-cpu-baseline > gpurun_out/lp_512.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_s256.so timeout -k 10 300 python3 -u bench.py --config loopburst --no-cpu-baseline > gpurun_out/lp_256.log 2>&1
echo LPDONE
