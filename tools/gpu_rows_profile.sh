# rocprofv3 kernel stats of the GPU parity tests of the rows outside the
# extraction stream (PnP, Sim3, BoW, projection/frustum, frame set-up, stereo,
# Initializer, loop burst): per-kernel durations at the tests' problem sizes.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rows_ks -o ks -- \
    python3 -m pytest -x -q -m gpu tests/test_pnp.py tests/test_ransac.py tests/test_bow.py tests/test_proj.py \
    tests/test_frame.py tests/test_stereo.py tests/test_init.py tests/test_loop.py tests/test_match_capacity.py > gpurun_out/rows_ks.log 2>&1
timeout -k 10 120 python3 tools/init_timing.py > gpurun_out/rows_init.log 2>&1
echo ALLDONE
