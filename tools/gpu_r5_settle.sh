# Round-5 diagnostic: the driver's command (--steps 20 --warmup 5, CPU legs off) with
# per-step GPU times, for each BENCH_SETTLE_STEPS value given in order (the first is the
# box's first bench process).   usage: bash tools/gpu_r5_settle.sh <tag> 20 0
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
i=0
for v in "$@"; do
  i=$((i + 1))
  BENCH_STEP_TRACE=1 BENCH_SETTLE_STEPS=$v timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_${i}_settle$v.log 2>&1
done
echo SETTLEDONE
