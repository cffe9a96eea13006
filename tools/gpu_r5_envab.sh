# Round-5 environment-knob A/B: for each value of $AB_VAR in $AB_VALS, the
# extraction parity tests under that value (test_gpu_parity.py, incl. the
# B = 512 headline batch), then the bench line (no extras / CPU legs, 40 timed
# steps after 20 warm-up steps) for every value, interleaved over $ROUNDS rounds.
# usage: AB_VAR=ORBGPU_OCT_SPLIT AB_VALS="0 64 128" ROUNDS=3 bash tools/gpu_r5_envab.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
for v in ${AB_VALS}; do
  env ${AB_VAR}=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par_${AB_VAR}${v}.log 2>&1
done
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${AB_VALS}; do
    env ${AB_VAR}=$v timeout -k 10 200 $B > gpurun_out/${tag}_${AB_VAR}${v}_$r.log 2>&1
  done
done
echo ENVABDONE
