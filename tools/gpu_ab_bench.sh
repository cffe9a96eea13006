# A/B: default library vs variants given as arguments (liborbgpu_<name>.so),
# bench without extras; one log per variant.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_base.log 2>&1
for v in "$@"; do
  ORBGPU_LIBRARY=$GRAFT_REPO_ROOT/orb-slam2-annotation_amd/liborbgpu_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_$v.log 2>&1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_base2.log 2>&1
echo DONE
