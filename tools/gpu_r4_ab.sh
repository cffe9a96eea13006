# A/B of the product library against variants (liborbgpu_<name>.so): extraction
# parity of each, then alternated bench lines (no extras / CPU legs), then the
# LDS / instruction PMC pass of each.  usage: bash tools/gpu_r4_ab.sh <tag> <variant>...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
L=$GRAFT_REPO_ROOT/orb-slam2-annotation_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par_base.log 2>&1
ok=""
for v in "$@"; do
  # a variant whose parity fails is reported and left out of the timing (a parity
  # failure is an ordinary test failure, not a GPU fault: the loop goes on)
  if ORBGPU_LIBRARY=$L/liborbgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par_$v.log 2>&1; then
    ok="$ok $v"
  else
    rc=$?
    echo "variant $v parity rc $rc"
    if [ $rc -ne 1 ]; then exit $rc; fi
  fi
done
set -- $ok
for rep in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --deliver gpu0 > gpurun_out/${tag}_base_$rep.log 2>&1
  for v in "$@"; do
    ORBGPU_LIBRARY=$L/liborbgpu_$v.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --deliver gpu0 > gpurun_out/${tag}_${v}_$rep.log 2>&1
  done
done
for pp in ${AB_LIGHT:+} "2 fast_cells 0" "2 fast_cells -1" "1 pyramid -1" "2 pyramid -1"; do
  [ -n "$AB_LIGHT" ] && break
  set -- $pp
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --deliver gpu0 --parts $1 --part-stage $2 --match-priority $3 > gpurun_out/${tag}_parts$1_$2_m$3.log 2>&1 || echo "parts $pp rc $?"
done
set -- $ok
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --deliver gpu0"
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES --output-format csv -d gpurun_out/${tag}_pmc_base -o q -- $B > gpurun_out/${tag}_pmc_base.log 2>&1
for v in "$@"; do
  ORBGPU_LIBRARY=$L/liborbgpu_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES --output-format csv -d gpurun_out/${tag}_pmc_$v -o q -- $B > gpurun_out/${tag}_pmc_$v.log 2>&1
done
echo ABDONE
if [ -z "$AB_LIGHT" ] && [ -f tools/split_probe.py ]; then
  timeout -k 10 300 python3 -u tools/split_probe.py > gpurun_out/${tag}_split.log 2>&1 || echo "split probe rc $?"
fi
echo SPLITDONE
if [ -z "$AB_LIGHT" ]; then
  timeout -k 10 400 bash tools/gpu_r4_dropin.sh ${tag} > gpurun_out/${tag}_dropin.log 2>&1 || echo "dropin rc $?"
fi
echo ABALLDONE
