# Pyramid tick variants (level-0 rows per tick, register budget): headline bench per library.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/pyr_base.log 2>&1
for v in t4 t4w t16; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_$v.so timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/pyr_$v.log 2>&1 || echo "variant $v failed rc=$?"
done
echo PYRDONE
