# FAST survivor-list cap (32 waves per CU) at HEAD: extraction parity (incl.
# the noise frame, whose cells overflow the list and take the all-pixel path),
# the matcher / adapter tests, then three default-line benches.
# usage: bash tools/gpu_r4_fastcap.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_adapter.py tests/test_match_capacity.py > gpurun_out/${tag}_par.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_bench_$rep.log 2>&1
done
echo FASTCAPDONE
