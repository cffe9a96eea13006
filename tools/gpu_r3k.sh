# Round-3 check k: extractor / BoW / loop / adapter / PnP parity, drop-in
# latencies, loop burst, PnP 16-solver batch timing (+ rocprofv3), headline.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3k}
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bow.py tests/test_loop.py tests/test_adapter.py tests/test_pnp.py tests/test_refpin.py tests/test_triangulation.py -m gpu -v -x --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -u tools/dropin_profile.py 40 > gpurun_out/${tag}_dropin.json 2> gpurun_out/${tag}_dropin.err
timeout -k 10 300 python3 -u bench.py --config loopburst --no-cpu-baseline > gpurun_out/${tag}_loop.log 2>&1
timeout -k 10 120 python3 -u tools/pnp_batch_timing.py 16 300 300 20 > gpurun_out/${tag}_pnp16.json 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_pnpks -o ks -- python3 tools/pnp_batch_timing.py 16 300 300 10 > gpurun_out/${tag}_pnpks.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo ALLDONE pytest_rc=$rc
