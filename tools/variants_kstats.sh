# GPU side: kernel-trace stats of every exp/*/liborbgpu.so variant (per-kernel average time).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in exp/*/; do
    n=$(basename $d)
    ORBGPU_LIBRARY=$PWD/$d/liborbgpu.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/vk_$n -o vk -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/vk_$n.log 2>&1
    python3 - "$n" gpurun_out/vk_$n/vk_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[2])) if "orbgpu" in r["Name"]]
print(sys.argv[1], " ".join(f"{r['Name'].split('::')[-1].split('(')[0][:18]}={float(r['AverageNs'])/1e3:.0f}" for r in rows))
PY
done
