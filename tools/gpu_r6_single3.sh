# Round-6 single-frame A/B over variants given as label:library[:ENV=V,ENV=V]:
# orbgpu_extract median (tools/single_frame_probe.py), interleaved over $ROUNDS
# rounds, then a kernel trace (timeline) and a kernel + HIP-runtime trace
# (host-side breakdown) of the first variant.
# usage: ROUNDS=3 bash tools/gpu_r6_single3.sh <tag> spec1 spec2 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
run_spec() {  # spec, then the command
  local spec=$1; shift
  local lib=$(echo "$spec" | cut -d: -f2) envs=$(echo "$spec" | cut -d: -f3)
  env ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so $(echo "$envs" | tr ',' ' ') "$@"
}
for r in $(seq 1 ${ROUNDS:-3}); do
  for spec in "$@"; do
    echo "$(echo $spec | cut -d: -f1) round $r" >> gpurun_out/${tag}_single.log
    run_spec "$spec" timeout -k 10 120 python3 -u tools/single_frame_probe.py >> gpurun_out/${tag}_single.log 2>&1 || { echo "probe $spec failed"; exit 3; }
  done
done
first=$1
lib=$(echo "$first" | cut -d: -f2)
envs=$(echo "$first" | cut -d: -f3 | tr ',' ' ')
for e in $envs; do export "$e"; done
ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 tools/single_frame_probe.py > gpurun_out/${tag}_ks.log 2>&1 || { echo "trace failed"; exit 3; }
ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/${tag}_host -o h -- python3 tools/single_frame_probe.py > gpurun_out/${tag}_host.log 2>&1 || { echo "host trace failed"; exit 3; }
python3 tools/single_frame_host.py gpurun_out/${tag}_host > gpurun_out/${tag}_host.txt 2>&1 || true
python3 tools/dropin_timeline.py gpurun_out/${tag}_ks --anchor pyramid_band --before 0 --after 3 > gpurun_out/${tag}_timeline.txt 2>&1 || true
echo SINGLE3DONE
