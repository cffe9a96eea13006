# Drop-in ORBextractor::operator() (tests/cpp/adapter_main extract, 640x480,
# 1000 features): the timed log, then the same run under a kernel + copy
# trace so each call's kernels, copies and the gaps between them can be read
# (tools/dropin_timeline.py).  usage: bash tools/gpu_r4_dropin.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1
D=gpurun_out/${tag}_dropin
mkdir -p $D
python3 -c "
import sys; sys.path.insert(0, 'orb-slam2-annotation_amd')
import synth
fr = synth.mono_stream(2, 640, 480)
for k in range(2): open('$D/f%d.raw' % k, 'wb').write(fr[k].tobytes())
"
X="tests/cpp/adapter_main extract 640 480 1000 $D/f0.raw $D/f1.raw $D/x.out"
ADAPTER_REPS=200 ADAPTER_TIME_LOG=$D/times.jsonl timeout -k 10 120 $X > $D/run.log 2>&1
ORBGPU_SINGLE_ZEROCOPY=0 ADAPTER_REPS=200 ADAPTER_TIME_LOG=$D/times_sdma.jsonl timeout -k 10 120 $X > $D/run_sdma.log 2>&1
ADAPTER_REPS=200 ADAPTER_TIME_LOG=$D/times_traced.jsonl timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace \
  --output-format csv -d $D/prof -o t -- $X > $D/prof.log 2>&1
echo DROPIN_DONE
