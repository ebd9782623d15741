# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit 1; }
for v in default; do
  if [ $v = default ]; then L=$PWD/flac-py_amd/libflacmi.so; else L=$PWD/flac-py_amd/libflacmi_$v.so; fi
  FLACMI_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-parity --e2e-units 0 --no-frames > $O/b_$v.json 2> $O/tr.err || { tail $O/tr.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/tr_$v/run_kernel_stats.csv')):
    if 'k_resid' in r['Name'] or 'k_lpc' in r['Name']: print('$v', r['Name'][:50], '%.3f' % (float(r['AverageNs'])/1e6))
"
done
