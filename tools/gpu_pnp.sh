# PnP / Initializer per-call check: parity tests, EPnP phase stamps (diagnostic
# build), drop-in latencies, kernel stats of the drop-in run.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-pnp}
timeout -k 10 300 python -u -m pytest tests/test_pnp.py tests/test_init.py tests/test_adapter.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_stamps.so timeout -k 10 120 python3 -u tools/epnp_stamps.py > gpurun_out/${tag}_stamps.txt 2>&1
timeout -k 10 300 python3 -u tools/dropin_profile.py 40 > gpurun_out/${tag}_dropin.json 2> gpurun_out/${tag}_dropin.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_dk -o dk_%pid% -- python3 tools/dropin_profile.py 10 > gpurun_out/${tag}_dk.log 2>&1
echo ALLDONE
