# Round-6 call 21: stereo kernel prefetching the next left keypoint (wave-uniform
# wave index): stereo / adapter / device
# tests, then the EuRoC and KITTI stereo configs, default vs HEAD (liborbgpu_base),
# and a kernel trace of each.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_stereo.py tests/test_adapter.py tests/test_devices.py > gpurun_out/r6z_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6z_tests.log; exit $rc; }
tail -1 gpurun_out/r6z_tests.log
for r in 1 2; do
  for lib in liborbgpu liborbgpu_base; do
    for cfg in euroc_stereo kitti_stereo; do
      ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 python3 -u bench.py --config $cfg --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/r6z_${cfg}_${lib}_$r.log 2>&1 || { echo "$cfg $lib failed"; exit 3; }
    done
  done
done
for lib in liborbgpu liborbgpu_base; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6z_ks_$lib -o ks -- python3 bench.py --config euroc_stereo --no-cpu-baseline --no-extras --steps 5 --warmup 2 > gpurun_out/r6z_ks_$lib.log 2>&1 || { echo "trace $lib failed"; exit 3; }
done
echo CALL21DONE
