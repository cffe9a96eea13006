# Round-6 call 29: extraction alone (tools/extract_iso.py, no matcher beside it)
# under rocprofv3 --kernel-trace --stats for the grouped MFMA describe (default),
# one slot per wave (liborbgpu_g1) and the VALU blur (liborbgpu_base).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6ah}
for lib in liborbgpu liborbgpu_g1 liborbgpu_base; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_$lib -o k -- python3 tools/extract_iso.py 512 30 > gpurun_out/${tag}_$lib.log 2>&1 || { echo "$lib failed"; exit 3; }
done
echo CALL29DONE
