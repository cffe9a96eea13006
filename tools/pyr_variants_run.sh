# GPU side: bench every exp/*/liborbgpu.so (pyramid stage time per variant).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in exp/*/; do
    n=$(basename $d)
    ORBGPU_LIBRARY=$PWD/$d/liborbgpu.so timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var_$n.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/var_$n.log').read().strip().splitlines()[-1]); print('$n', d['stages_ms_per_step'], d['parity_frame0_vs_oracle'])"
done
