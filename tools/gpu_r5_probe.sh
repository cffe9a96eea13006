# Round-5 latency probes: the bench line with the product library and with
# diagnostic builds (FAST windows / describe neighbourhoods all from frame 0:
# L2-resident), then the phase stamps of the -DFAST_STAMPS -DDESC_STAMPS build.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
for lib in liborbgpu liborbgpu_pf liborbgpu_pd; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20 > gpurun_out/${tag}_bench_$lib.log 2>&1 || echo "$lib failed"
done
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xs.so timeout -k 10 200 python3 tools/extract_stamps.py > gpurun_out/${tag}_stamps.json 2>&1 || echo "stamps failed"
echo PROBEDONE
