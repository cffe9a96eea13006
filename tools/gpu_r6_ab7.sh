# Round-6 call 7: the banded (single-frame) pyramid with its resize tables staged
# in LDS: pyramid / adapter parity, then single-frame latency against the build
# without the staging (notab).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6h}
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_adapter.py tests/test_stereo.py > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; exit $rc; }
ROUNDS=3 bash tools/gpu_r6_single.sh ${tag} liborbgpu liborbgpu_notab
echo AB7DONE
