# Stereo drop-in tail: the stereo Frame of tests/cpp/adapter_main
# (two ORBextractor threads + ComputeStereoMatches, 752x480 / 1200 features)
# timed over $REPS repetitions twice, with the attribution rows (thread pair
# alone, both extractions on one thread), then once under a kernel trace so the
# slow calls' GPU time can be told from their host time (tools/dropin_timeline.py).
# usage: REPS=1000 bash tools/gpu_r5_stereo.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1
D=gpurun_out/${tag}_stereo
mkdir -p $D
python3 -c "
import sys; sys.path.insert(0, 'orb-slam2-annotation_amd')
import numpy as np, synth
st = synth.stereo_stream(1, 752, 480, 0x5E7, 18.0)[0]
open('$D/l.raw', 'wb').write(st[0].tobytes()); open('$D/r.raw', 'wb').write(st[1].tobytes())
"
BF=$(python3 -c "import numpy as np; print(repr(float(np.float32(47.90639384423901))))")
X="tests/cpp/adapter_main stereo 752 480 1200 $BF $D/l.raw $D/r.raw $D/x.out"
for k in 1 2; do
  ADAPTER_REPS=${REPS:-1000} ADAPTER_TIME_LOG=$D/times_$k.jsonl timeout -k 10 180 $X > $D/run_$k.log 2>&1
done
ADAPTER_REPS=300 ADAPTER_TIME_LOG=$D/times_traced.jsonl timeout -k 10 180 rocprofv3 --kernel-trace \
  --output-format csv -d $D/prof -o t -- $X > $D/prof.log 2>&1
echo STEREODONE
