# Matcher placement after the octree LDS change: the bench line (no extras / CPU legs,
# 40 timed steps after 20 warm-up steps) with --match-after fast_cells / octree and the
# matcher stream at high priority, interleaved over $ROUNDS rounds.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-3}); do
  timeout -k 10 200 $B > gpurun_out/${tag}_fast_$r.log 2>&1
  timeout -k 10 200 $B --match-after octree > gpurun_out/${tag}_octree_$r.log 2>&1
  timeout -k 10 200 $B --match-priority -1 > gpurun_out/${tag}_fastprio_$r.log 2>&1
done
echo PLACEDONE
