# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_decode.py tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -60; exit 1; }
for v in default head default head; do
  if [ $v = default ]; then L=$PWD/flac-py_amd/libflacmi.so; else L=$PWD/flac-py_amd/libflacmi_$v.so; fi
  FLACMI_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-parity > $O/b_$v.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); fw=d['frame_writer']; print('$v', 'frames ms %.3f' % fw['ms_per_call'])"
done
