# PMC passes over the bench (pyramid_kernel analysis); each pass separate.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/q1 -o q1 -- $B > gpurun_out/q1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/q2 -o q2 -- $B > gpurun_out/q2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/q1/q1_counter_collection.csv gpurun_out/q2/q2_counter_collection.csv > gpurun_out/pmc_summary.txt
echo PMCDONE
