# Round-3 check b: Initializer / PnP / adapter / parity GPU tests, then the
# drop-in latencies plain and under rocprofv3 kernel stats.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3b}
rc=0
timeout -k 10 600 python -u -m pytest tests/test_init.py tests/test_pnp.py tests/test_adapter.py tests/test_gpu_parity.py tests/test_ransac.py -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -u tools/dropin_profile.py 40 > gpurun_out/${tag}_dropin.json 2> gpurun_out/${tag}_dropin.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_dk -o dk -- python3 tools/dropin_profile.py 10 > gpurun_out/${tag}_dk.log 2>&1
echo ALLDONE pytest_rc=$rc
