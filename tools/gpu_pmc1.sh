# Extractor parity, one instruction-mix PMC pass over the mono640 step, and
# the headline bench line (stage times).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-p1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/${tag}_1 -o q -- $B > gpurun_out/${tag}_1.log 2>&1
python3 tools/pmc_summary.py gpurun_out/${tag}_1/q_counter_collection.csv > gpurun_out/${tag}_pmc_summary.txt 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo PMC1DONE
