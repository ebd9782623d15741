# GPU suite, then the frame-writer leg (config 2, 1e6 frames) of this build against
# flac-py_amd/libflacmi_r04base.so, alternating on one box.  Usage: bash tools/gpu_frames_ab.sh <tag>
set -o pipefail
TAG=${1:-frames_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
BASE=$PWD/flac-py_amd/libflacmi_r04base.so
for v in new base new base; do
  if [ $v = base ]; then export FLACMI_LIB=$BASE; else unset FLACMI_LIB; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity --e2e-units 0 > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail -20 $OUT/c2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_$v.json'));print('$v', 'frame_ms %.3f' % d['frame_writer']['ms_per_call'], 'value %.4e' % d['value'])"
done
unset FLACMI_LIB
