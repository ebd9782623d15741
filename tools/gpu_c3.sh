# gpu parity tests, then the c3 bench line (24-bit stereo, L=32 q=15) and its kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --no-parity --no-frames > /dev/null 2> gpurun_out/prof_c3.err || { tail gpurun_out/prof_c3.err; exit 1; }
head -8 gpurun_out/prof_c3/run_kernel_stats.csv | cut -c1-160
