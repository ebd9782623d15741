# Round-3 iteration: GPU suite, smoke, c2 bench with and without LPC pruning.
# Usage: bash tools/gpu_r03.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r03}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 2 --e2e-units 0 --no-frames "$@" > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python tools/show_bench.py $OUT/bench_c2.json
FLACMI_NO_PRUNE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e-units 0 --no-frames "$@" > $OUT/bench_c2_noprune.json 2> $OUT/bench_c2_noprune.err || { tail -20 $OUT/bench_c2_noprune.err; exit 1; }
python tools/show_bench.py $OUT/bench_c2_noprune.json
