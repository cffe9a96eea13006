# Round-6 single-frame A/B: orbgpu_extract (the drop-in path) median latency
# for each library named, interleaved over $ROUNDS rounds, then a kernel
# trace + stats of the probe per library (per-kernel durations of one call).
# usage: ROUNDS=3 bash tools/gpu_r6_single.sh <tag> lib1 lib2 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in "$@"; do
    echo "$lib round $r" >> gpurun_out/${tag}_single.log
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 120 python3 -u tools/single_frame_probe.py >> gpurun_out/${tag}_single.log 2>&1 || { echo "$lib failed"; exit 3; }
  done
done
for lib in "$@"; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks_${lib} -o ks -- python3 tools/single_frame_probe.py > gpurun_out/${tag}_ks_${lib}.log 2>&1 || { echo "trace $lib failed"; exit 3; }
done
echo SINGLEDONE
