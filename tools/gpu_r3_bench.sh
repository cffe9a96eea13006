# Round-3 bench call: PMC passes at HEAD over the mono640 step (instruction
# mix, waits, LDS, HBM FETCH/WRITE -> pmc_traffic.json), the full default
# bench line with that traffic, and rocprofv3 kernel stats of a short bench.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3bench}
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/${tag}_1 -o q -- $B > gpurun_out/${tag}_1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/${tag}_2 -o q -- $B > gpurun_out/${tag}_2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/${tag}_4 -o q -- $B > gpurun_out/${tag}_4.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_f -o q -- $B > gpurun_out/${tag}_f.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_w -o q -- $B > gpurun_out/${tag}_w.log 2>&1
python3 tools/pmc_summary.py gpurun_out/${tag}_1/q_counter_collection.csv gpurun_out/${tag}_2/q_counter_collection.csv gpurun_out/${tag}_4/q_counter_collection.csv gpurun_out/${tag}_f/q_counter_collection.csv gpurun_out/${tag}_w/q_counter_collection.csv > gpurun_out/${tag}_pmc_summary.txt 2>&1
python3 tools/make_traffic.py gpurun_out/${tag}_f/q_counter_collection.csv gpurun_out/${tag}_w/q_counter_collection.csv --config mono640 --batch 512 --algorithmic 803777536 --out gpurun_out/${tag}_pmc_traffic.json > gpurun_out/${tag}_traffic.log 2>&1
timeout -k 10 600 python3 -u bench.py --traffic-json gpurun_out/${tag}_pmc_traffic.json > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_ks.log 2>&1
echo ALLDONE
