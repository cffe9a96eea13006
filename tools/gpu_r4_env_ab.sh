# Parity tests matching -k PATTERN, then alternated default-line benches (no
# CPU legs, no extras) with the environment variable VAR set to each value.
# usage: bash tools/gpu_r4_env_ab.sh <tag> <pytest -k pattern> <VAR> <value>...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; pat=$2; var=$3; shift 3
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$pat" > gpurun_out/${tag}_par.log 2>&1
for rep in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_${v}_$rep.log 2>&1
  done
done
echo ENVABDONE
