# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bench" > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -60; exit 1; }
for c in c2 c3 c5; do timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-frames > $O/b_$c.json 2> $O/err_$c.txt || { tail $O/err_$c.txt; exit 1; }; python3 -c "import json; d=json.load(open('$O/b_$c.json')); print('$c', json.dumps(d['parity']))"; done
