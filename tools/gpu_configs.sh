# bench lines for the other BASELINE configs (c3 stereo 24-bit, c4 chunked 1e8 blocks, c5 fixed-only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail gpurun_out/bench_c5.err; exit 1; }
echo c5; cat gpurun_out/bench_c5.json
timeout -k 10 400 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
echo c3; cat gpurun_out/bench_c3.json
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail gpurun_out/bench_c4.err; exit 1; }
echo c4; cat gpurun_out/bench_c4.json
