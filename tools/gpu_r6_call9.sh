# Round-6 call 9 + single-frame breakdown in one box.
set -e
bash tools/gpu_r6_ab9.sh r6j
bash tools/gpu_r6_single2.sh r6k
