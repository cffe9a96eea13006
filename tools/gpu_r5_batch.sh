# Round-5 batch-size probe: the bench line (no extras / CPU legs, 40 timed steps
# after 20 warm-up steps) at B = 512, 1024 and 2048 frames per step, 2 rounds.
# usage: bash tools/gpu_r5_batch.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
for r in 1 2; do
  for b in ${BATCHES:-512 1024 2048}; do
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20 --batch $b > gpurun_out/${tag}_batch${b}_$r.log 2>&1
  done
done
echo BATCHDONE
