# int8-MFMA candidate sums (PATH_W64): GPU tests, then c3 bench lines with the MFMA path
# and with FLACMI_NO_MFMA=1 (the v_mad_i64_i32 chains) for comparison.
# Usage: bash tools/gpu_mf8.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-mf8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --no-frames > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3',d['value'],d['kernels'],d['roofline']['frac'],d['parity'])"
FLACMI_NO_MFMA=1 timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --no-frames > $OUT/bench_c3_nomfma.json 2> $OUT/bench_c3_nomfma.err || { tail -20 $OUT/bench_c3_nomfma.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c3_nomfma.json'));print('c3 no-mfma',d['value'],d['kernels'],d['roofline']['frac'],d['parity'])"
