# full GPU suite, then the c3 line under rocprofv3 kernel stats
set -o pipefail
TAG=${1:-r02c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --no-frames --e2e-units 0 > $OUT/bench_c3_under_rocprof.json 2> $OUT/prof_c3.err || { tail $OUT/prof_c3.err; exit 1; }
head -6 $OUT/prof_c3/run_kernel_stats.csv | cut -c1-200
