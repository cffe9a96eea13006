# PMC passes over the whole mono640 step (every kernel): SQ instruction mix and
# wave-cycle split, busy/clock, TA/TCP, HBM FETCH/WRITE; one pass per set.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r2pmc}
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/${tag}_1 -o q -- $B > gpurun_out/${tag}_1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/${tag}_2 -o q -- $B > gpurun_out/${tag}_2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/${tag}_3 -o q -- $B > gpurun_out/${tag}_3.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/${tag}_4 -o q -- $B > gpurun_out/${tag}_4.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_f -o q -- $B > gpurun_out/${tag}_f.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_w -o q -- $B > gpurun_out/${tag}_w.log 2>&1
python3 tools/pmc_summary.py gpurun_out/${tag}_1/q_counter_collection.csv gpurun_out/${tag}_2/q_counter_collection.csv gpurun_out/${tag}_3/q_counter_collection.csv gpurun_out/${tag}_4/q_counter_collection.csv gpurun_out/${tag}_f/q_counter_collection.csv gpurun_out/${tag}_w/q_counter_collection.csv > gpurun_out/${tag}_summary.txt 2>&1
echo ALLDONE
