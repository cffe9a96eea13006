# FAST/describe iteration on the GPU box: extraction parity, PMC of the
# extraction kernels, kernel stats of a short bench.  usage: bash tools/gpu_fast_iter.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fast}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_ks.log 2>&1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/${tag}_1 -o q -- $B > gpurun_out/${tag}_1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${tag}_2 -o q -- $B > gpurun_out/${tag}_2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/${tag}_1/q_counter_collection.csv gpurun_out/${tag}_2/q_counter_collection.csv > gpurun_out/${tag}_summary.txt 2>&1
echo ALLDONE
