# Round-6 call 11: the whole -m gpu suite on the default build (single-frame upload
# fused into the band pyramid, 64 bands), the single-frame parity tests again with
# the streamed upload (ORBGPU_SINGLE_STREAMED=1), then the single-frame A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6m_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6m_tests.log; exit $rc; }
tail -2 gpurun_out/r6m_tests.log
ORBGPU_SINGLE_STREAMED=1 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "single_frame or extract" tests/test_adapter.py > gpurun_out/r6m_streamed_tests.log 2>&1 || { rc=$?; echo "streamed tests rc=$rc"; tail -30 gpurun_out/r6m_streamed_tests.log; exit $rc; }
tail -2 gpurun_out/r6m_streamed_tests.log
ROUNDS=3 bash tools/gpu_r6_single3.sh r6m new:liborbgpu head:liborbgpu_base new_spin:liborbgpu:ORBGPU_SINGLE_WAIT=1 \
  new_nofuse:liborbgpu:ORBGPU_SINGLE_FUSED_UPLOAD=0 new_b96:liborbgpu:ORBGPU_PYR_BANDS_MAX=96 \
  new_stream:liborbgpu:ORBGPU_SINGLE_STREAMED=1 new_stream_spin:liborbgpu:ORBGPU_SINGLE_STREAMED=1,ORBGPU_SINGLE_WAIT=1
ROUNDS=0 bash tools/gpu_r6_single3.sh r6m_st new_stream_spin:liborbgpu:ORBGPU_SINGLE_STREAMED=1,ORBGPU_SINGLE_WAIT=1
echo CALL11DONE
