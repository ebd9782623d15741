# Iteration check on the GPU box: GPU suite, c2 bench line, rocprofv3 kernel stats of c2.
# Usage: bash tools/gpu_iter.sh <tag> [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-iter}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e-units 0 --no-frames "$@" > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python tools/show_bench.py $OUT/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-parity --e2e-units 0 --no-frames "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("$OUT/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:8]:
    print("%-60s calls %6s avg %.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
