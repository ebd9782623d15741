# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ls; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "frame or decode or writer or cli or encoder" > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
for spec in c3:5:1 c3:5:0 c3:8:1 c3:0:1 c2:5:1; do
  c=${spec%%:*}; r=${spec#*:}; k=${r%%:*}; l=${r##*:}
  FLACMI_DECODE_LPC=$l timeout -k 10 300 python bench.py --config $c --open $k --steps 1 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-parity > $O/b_${c}_${k}_$l.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_${c}_${k}_$l.json')); f=d['frame_writer']; r=f['decoder_round_trip']; print('$spec', 'decode', round(r['ms_per_call'],2), r['frames_with_status'], r['samples_mismatched'], 'pack', round(f['ms_per_call'],2))"
done
