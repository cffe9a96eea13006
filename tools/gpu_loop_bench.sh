# parity subset, default bench, loop-burst bench + its rocprof summary
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r2d}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_frame.py > gpurun_out/${tag}_par.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 300 python -u bench.py --config loopburst > gpurun_out/${tag}_loop.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_loopks -o ks -- python3 bench.py --config loopburst --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_loopks.log 2>&1
echo ALLDONE
