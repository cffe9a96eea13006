# Round-5 diagnostic: the driver's command (--steps 20 --warmup 5, CPU legs off) once per
# BENCH_PROF_STEPS value given, in order (-1: stage events on every timed step, the
# default; 1: on the last step only).   usage: bash tools/gpu_r5_profab.sh <tag> -1 1 -1 1
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
i=0
for v in "$@"; do
  i=$((i + 1))
  BENCH_PROF_STEPS=$v timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_${i}_prof$v.log 2>&1
done
echo PROFABDONE
