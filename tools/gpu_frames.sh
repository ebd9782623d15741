set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_frames.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_frames.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --units 200000 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_frames.json 2> gpurun_out/bench_frames.err || { echo bench failed; tail -30 gpurun_out/bench_frames.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_frames.json')); print(d['value'], d['kernels']['k_resid_ms']); print(json.dumps(d['frame_writer']))"
