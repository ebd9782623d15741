# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "production or overlap or async or stream or lds" > $O/pt.log 2>&1; rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --e2e-units 0 --no-frames --parity-units 32"
for spec in "c2:0" "c2:5" "c2:8" "c2:0"; do
  c=${spec%%:*}; k=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --open $k $B > $O/b_${c}_o$k.json 2> $O/e_${c}_o$k.txt || { tail $O/e_${c}_o$k.txt; exit 1; }
  python -c "import json;d=json.load(open('$O/b_${c}_o$k.json'));print('$c o$k',d['value'],d['kernels']['k_resid_ms'],d['kernels']['k_lpc_ms'],d['roofline']['frac'],(d.get('parity') or {}).get('mismatches'))"
done
