set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_frames.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_frames.log
