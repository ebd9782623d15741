# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r7g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "overlap" > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
for v in cur head cur head; do
  L=$PWD/flac-py_amd/libflacmi.so
  [ $v = head ] && L=$PWD/flac-py_amd/libflacmi_head.so
  FLACMI_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-frames > $O/b_$v.json 2> $O/err_$v.txt || { tail $O/err_$v.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); e=d['end_to_end']; print('$v', d['ms_per_step'], d['value'], e['wall_ms'])"
  FLACMI_LIB=$L timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0 > $O/b3_$v.json 2> $O/err3_$v.txt || { tail $O/err3_$v.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b3_$v.json')); print('$v c3', d['ms_per_step'], d['value'])"
done
