# Round-5 iteration call: extraction/match parity (+ extra test files given), a
# bench line without extras / CPU legs, and the kernel trace + stats of a short
# bench (per-launch durations: tools/ks_top.py, tools/pyr_launches.py).
# usage: bash tools/gpu_r5_iter.sh <tag> [test files...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py "$@" > gpurun_out/${tag}_par.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_ks.log 2>&1
echo ITERDONE
