set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --units 200000 --steps 5 --warmup 2 --cpu-seconds 3 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || { echo "bench_small failed"; tail -20 gpurun_out/bench_small.err; exit 1; }
cat gpurun_out/bench_small.json
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o run -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity > gpurun_out/prof_r1.log 2>&1; echo "rocprof rc=$?"
find gpurun_out/prof_r1 -name "*stats*" | head
