# Round-3 check m: extractor / BoW / loop / adapter parity, drop-in
# latencies (+ per-process rocprofv3), loop burst, headline.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3m}
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bow.py tests/test_loop.py tests/test_adapter.py tests/test_refpin.py -m gpu -v -x --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -u tools/dropin_profile.py 40 > gpurun_out/${tag}_dropin.json 2> gpurun_out/${tag}_dropin.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_dk -o dk_%pid% -- python3 tools/dropin_profile.py 10 > gpurun_out/${tag}_dk.log 2>&1
timeout -k 10 300 python3 -u bench.py --config loopburst --no-cpu-baseline > gpurun_out/${tag}_loop.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo ALLDONE pytest_rc=$rc
