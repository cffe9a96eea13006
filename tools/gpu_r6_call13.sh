# Round-6 call 13: single-frame host path variants -- completion flag (default)
# vs hipStreamSynchronize, each with the pinned staging + copy kernel (default)
# or the host writing the frame straight into host-mapped fine-grained HBM
# (ORBGPU_SINGLE_VRAM_STAGING=1): the single-frame parity tests with the latter,
# then the python probe and the C++ drop-in class, interleaved.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ORBGPU_SINGLE_VRAM_STAGING=1 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "single_frame or extract" tests/test_adapter.py > gpurun_out/r6p_vram_tests.log 2>&1 || { rc=$?; echo "vram tests rc=$rc"; tail -30 gpurun_out/r6p_vram_tests.log; exit $rc; }
tail -1 gpurun_out/r6p_vram_tests.log
ROUNDS=3 bash tools/gpu_r6_single3.sh r6p flag:liborbgpu sync:liborbgpu:ORBGPU_SINGLE_DONE_FLAG=0 \
  vram:liborbgpu:ORBGPU_SINGLE_VRAM_STAGING=1 vram_sync:liborbgpu:ORBGPU_SINGLE_VRAM_STAGING=1,ORBGPU_SINGLE_DONE_FLAG=0
ROUNDS=3 REPS=1000 timeout -k 10 600 python3 -u tools/extract_cpp_probe.py flag sync=ORBGPU_SINGLE_DONE_FLAG=0 \
  vram=ORBGPU_SINGLE_VRAM_STAGING=1 vram_sync=ORBGPU_SINGLE_VRAM_STAGING=1,ORBGPU_SINGLE_DONE_FLAG=0 > gpurun_out/r6p_cpp.txt 2>&1 || { echo "cpp probe failed"; tail gpurun_out/r6p_cpp.txt; exit 3; }
cat gpurun_out/r6p_cpp.txt
echo CALL13DONE
