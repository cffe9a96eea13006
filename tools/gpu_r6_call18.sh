# Round-6 call 18: the pyramid tick plan with a larger compute-lane budget
# (ORBGPU_PYR_LANES_RT: more row groups, shorter per-tick maxima; CPU model
# tools/pyr_plan_cost.py): pyramid / extraction parity with 896 lanes, then the
# bench A/B over budgets 576 (default), 768, 896, 960.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ORBGPU_PYR_LANES_RT=896 timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r6w_parity896.log 2>&1 || { rc=$?; echo "parity rc=$rc"; tail -20 gpurun_out/r6w_parity896.log; exit $rc; }
tail -1 gpurun_out/r6w_parity896.log
ROUNDS=3 bash tools/gpu_r6_envab.sh r6w l576 l768=ORBGPU_PYR_LANES_RT=768 l896=ORBGPU_PYR_LANES_RT=896 l960=ORBGPU_PYR_LANES_RT=960
echo CALL18DONE
