# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "production or async or overlap or stream_constant" > $O/pt.log 2>&1; rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --e2e-units 0 --no-frames --parity-units 32"
for spec in "c2:0" "c2:5"; do
  c=${spec%%:*}; k=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --open $k $B > $O/b_${c}_o$k.json 2> $O/e_${c}_o$k.txt || { tail $O/e_${c}_o$k.txt; exit 1; }
  python tools/show_bench.py $O/b_${c}_o$k.json
done
FLACMI_NO_PRUNE=1 timeout -k 10 300 python bench.py --config c2 --open 5 $B > $O/b_c2_o5_np.json 2> $O/e_c2_o5_np.txt || { tail $O/e_c2_o5_np.txt; exit 1; }
python tools/show_bench.py $O/b_c2_o5_np.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c2 --open 5 --steps 3 --warmup 1 --cpu-seconds 0 --no-parity --e2e-units 0 --no-frames > $O/bench_trace.json 2> $O/trace.err || { tail $O/trace.err; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("$O/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:10]:
    print("%-70s calls %6s avg %.3f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
