# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r7e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "overlap or production or pruning or stream_constant" > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 --e2e-units 0 --no-frames > $O/b_$c.json 2> $O/err_$c.txt || { tail $O/err_$c.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['pipeline_frac'], json.dumps(d['kernels']), d['parity']['mismatches'])"
done
