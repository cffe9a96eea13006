# The driver's command (bench.py --gpus 1 --steps 20 --warmup 5, the full default line)
# $ROUNDS times, each line to gpurun_out/<tag>_line_<r>.log.   usage: ROUNDS=2 bash tools/gpu_r5_headline.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 ${EXTRA_ARGS} > gpurun_out/${tag}_line_$r.log 2>&1
done
echo HEADLINEDONE
