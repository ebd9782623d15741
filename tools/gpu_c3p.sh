# c3 iteration: GPU suite, c3 bench with and without LPC pruning.
set -o pipefail
TAG=${1:-c3p}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --cpu-seconds 0 --e2e-units 0 --no-frames > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
python tools/show_bench.py $OUT/bench_c3.json
FLACMI_NO_PRUNE=1 timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --cpu-seconds 0 --e2e-units 0 --no-frames > $OUT/bench_c3_noprune.json 2> $OUT/bench_c3_noprune.err || { tail -20 $OUT/bench_c3_noprune.err; exit 1; }
python tools/show_bench.py $OUT/bench_c3_noprune.json
