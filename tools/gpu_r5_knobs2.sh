# Knob A/B after the matcher/octree occupancy change: the bench line (no extras /
# CPU legs, 40 timed steps after 20 warm-up steps), interleaved over $ROUNDS rounds.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 $B > gpurun_out/${tag}_default_$r.log 2>&1
  ORBGPU_MATCH_THREADS=512 timeout -k 10 200 $B > gpurun_out/${tag}_mt512_$r.log 2>&1
  timeout -k 10 200 $B --match-after octree > gpurun_out/${tag}_afteroct_$r.log 2>&1
  ORBGPU_OCT_KCAP_A=1536 timeout -k 10 200 $B > gpurun_out/${tag}_kcap1536_$r.log 2>&1
done
echo KNOBS2DONE
