# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "c3 or mf8 or int8 or production or every_order or golden" > $O/pt.log 2>&1; rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -60; exit 1; }
for s in 1 2 4 5 6 7 0; do
  FLACMI_DEBUG_STOP=$s timeout -k 10 200 python bench.py --config c3 --steps 5 --warmup 2 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0 > $O/c3_s$s.json 2> $O/err || { tail $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/c3_s$s.json'));print('stop $s', '%.3f'%d['kernels']['k_resid_ms'])"
done
STOPS="2 0" KPAT=k_resid_sb UNITS=40000 bash tools/pmc_stops.sh r5f/pmc insts --config c3 --e2e-units 0 | grep -E "==|VALU|SALU|LDS"
