# Round-6 environment A/B on the default library: for each variant
# label=ENV=V[,ENV=V] (label alone: the environment as is), the bench line (no
# extras / CPU legs, 40 timed steps after 20 warm-up steps) interleaved over
# $ROUNDS rounds.   usage: ROUNDS=3 bash tools/gpu_r6_envab.sh <tag> spec1 spec2 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for r in $(seq 1 ${ROUNDS:-3}); do
  for spec in "$@"; do
    label=${spec%%=*}; envs=""; [ "$label" != "$spec" ] && envs=${spec#*=}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20 > gpurun_out/${tag}_${label}_$r.log 2>&1 || { echo "$label failed"; exit 3; }
  done
done
echo ENVABDONE
