# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6mf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "c3 or mf8 or sb or sign or production or open" > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
for v in new old new old; do
  E=""; [ $v = old ] && E="FLACMI_MF8_LIST=0"
  env $E timeout -k 10 300 python bench.py --config c3 --open 5 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-frames > $O/b_$v.json 2> $O/err_$v.txt || { tail $O/err_$v.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', d['value'], d['ms_per_step'], d['kernels']['k_resid_ms'], (d.get('parity') or {}).get('mismatches'), d['stream_stats']['lpc_tiers'], d['stream_stats']['lpc'])"
done
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-frames > $O/b_c3.json 2> $O/err_c3.txt && python3 -c "import json; d=json.load(open('$O/b_c3.json')); print('c3', d['value'], d['kernels']['k_resid_ms'], (d.get('parity') or {}).get('mismatches'))"
