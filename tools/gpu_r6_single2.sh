# Round-6 single-frame breakdown: orbgpu_extract median latency with the band
# pyramid capped at 32 (default), 48 and 64 bands (interleaved, 3 rounds), then a
# kernel + HIP-runtime trace of the default probe (host-side breakdown:
# tools/single_frame_host.py) and kernel stats per band count.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6k}
for r in 1 2 3; do
  for nb in 32 48 64; do
    echo "bands $nb round $r" >> gpurun_out/${tag}_single.log
    ORBGPU_PYR_BANDS_MAX=$nb timeout -k 10 120 python3 -u tools/single_frame_probe.py >> gpurun_out/${tag}_single.log 2>&1 || { echo "probe $nb failed"; exit 3; }
  done
done
for nb in 32 64; do
  ORBGPU_PYR_BANDS_MAX=$nb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks_$nb -o ks -- python3 tools/single_frame_probe.py > gpurun_out/${tag}_ks_$nb.log 2>&1 || { echo "trace $nb failed"; exit 3; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/${tag}_host -o h -- python3 tools/single_frame_probe.py > gpurun_out/${tag}_host.log 2>&1 || { echo "host trace failed"; exit 3; }
python3 tools/single_frame_host.py gpurun_out/${tag}_host > gpurun_out/${tag}_host.txt 2>&1 || true
python3 tools/dropin_timeline.py gpurun_out/${tag}_ks_32 --anchor copy16 --before 0 --after 4 > gpurun_out/${tag}_timeline_32.txt 2>&1 || true
python3 tools/dropin_timeline.py gpurun_out/${tag}_ks_64 --anchor copy16 --before 0 --after 4 > gpurun_out/${tag}_timeline_64.txt 2>&1 || true
echo SINGLE2DONE
