# Round-5 A/B call: parity (+ extra test files given), then the bench line
# (no extras / CPU legs) under each value of $AB_VAR listed in $AB_VALS, then
# rocprofv3 kernel trace + stats of a short default bench.
# usage: AB_VAR=ORBGPU_DESC_LEVEL_BLUR AB_VALS="0 2 3" bash tools/gpu_r5_ab.sh <tag> [test files...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py "$@" > gpurun_out/${tag}_par.log 2>&1
for v in ${AB_VALS:-default}; do
  if [ "$v" = default ]; then
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_bench_default.log 2>&1
  else
    env ${AB_VAR}=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_bench_${v}.log 2>&1
  fi
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_ks.log 2>&1
echo ABDONE
