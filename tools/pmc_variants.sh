# GPU side: SQ counter passes (pyramid analysis) for every exp/* variant.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for d in exp/*/; do
    n=$(basename $d)
    export ORBGPU_LIBRARY=$PWD/$d/liborbgpu.so
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/p1_$n -o q1 -- $B > gpurun_out/p1_$n.log 2>&1
    timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/p2_$n -o q2 -- $B > gpurun_out/p2_$n.log 2>&1
    echo "== $n" >> gpurun_out/pmc_variants.txt
    python3 tools/pmc_summary.py gpurun_out/p1_$n/q1_counter_collection.csv gpurun_out/p2_$n/q2_counter_collection.csv | grep -A30 "^pyramid" | head -26 >> gpurun_out/pmc_variants.txt
done
bash tools/variants_kstats.sh
