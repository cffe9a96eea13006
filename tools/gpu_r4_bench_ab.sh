# Alternated default-line benches (no CPU legs, no extras) of the product
# library under several bench.py argument sets; the first set is the base.
# usage: bash tools/gpu_r4_bench_ab.sh <tag> "<args of set 0>" "<args of set 1>" ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for rep in 1 2; do
  i=0
  for a in "$@"; do
    echo "set $i: $a" > gpurun_out/${tag}_s${i}_$rep.log
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras $a >> gpurun_out/${tag}_s${i}_$rep.log 2>&1 || echo "set $i rc $?"
    i=$((i + 1))
  done
done
echo BENCHABDONE
