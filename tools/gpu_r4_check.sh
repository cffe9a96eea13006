# Quick check of the product library: the extractor parity tests, then two
# default-line benches (no CPU legs, no extras).  usage: bash tools/gpu_r4_check.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_bench_$rep.log 2>&1
done
echo CHECKDONE
