# Round-2 iteration on the GPU box: GPU tests, smoke, a c2 and a c5 bench line.
# Usage: bash tools/gpu_r02.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r02}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --cpu-seconds 2 --no-frames $* > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));print('c2',d['value'],d['kernels'],d['roofline']['frac'],d['parity'])"
timeout -k 10 300 python bench.py --config c5 --cpu-seconds 0 --no-frames $* > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c5.json'));print('c5',d['value'],d['kernels'],d['roofline']['frac'],d['parity'])"
