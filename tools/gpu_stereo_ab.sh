# Stereo split A/B: stereo parity, then drop-in latencies at several block splits.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stereo.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/st_gpu.log 2>&1
for s in 8 16 32 64; do
  ORBGPU_STEREO_SPLIT_MAX=$s timeout -k 10 300 python3 -u tools/dropin_profile.py 20 > gpurun_out/st_dropin_$s.json 2> gpurun_out/st_dropin_$s.err
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/st_bench.log 2>&1
echo STDONE
