# GPU side: SQ counter passes for the pyramid kernel, frame and band modes.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
rm -f gpurun_out/pmc_modes.txt
for m in ${MODES:-frame band}; do
    export ORBGPU_PYR_MODE=$m
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/m1_$m -o q1 -- $B > gpurun_out/m1_$m.log 2>&1
    timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/m2_$m -o q2 -- $B > gpurun_out/m2_$m.log 2>&1
    timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/m3_$m -o q3 -- $B > gpurun_out/m3_$m.log 2>&1 || true
    echo "== $m" >> gpurun_out/pmc_modes.txt
    python3 tools/pmc_summary.py gpurun_out/m1_$m/q1_counter_collection.csv gpurun_out/m2_$m/q2_counter_collection.csv $(ls gpurun_out/m3_$m/q3_counter_collection.csv 2>/dev/null) | grep -A34 "^pyramid" | head -32 >> gpurun_out/pmc_modes.txt
done
