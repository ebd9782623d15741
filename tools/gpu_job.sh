# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6za; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "frame or writer or cli or encoder or decode" > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
for v in cur pre cur pre; do
  L=$PWD/flac-py_amd/libflacmi.so
  [ $v = pre ] && L=$PWD/flac-py_amd/libflacmi_pre.so
  FLACMI_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --e2e-units 0 > $O/b_$v.json 2> $O/err_$v.txt || { tail $O/err_$v.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); f=d['frame_writer']; r=f['decoder_round_trip']; print('$v pack', round(f['ms_per_call'],3), 'decode', round(r['ms_per_call'],3), r['frames_with_status'], r['samples_mismatched'], f['parity']['mismatches'])"
done
