# Round checkpoint: GPU suite, smoke, default bench line, rocprof trace + FETCH/WRITE for c2, c3
# and c5, bench lines for c3/c4/c5.  Usage: bash tools/gpu_round_ckpt.sh <tag>
set -o pipefail
TAG=${1:-ckpt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python tools/show_bench.py $OUT/bench_c2.json 2>/dev/null || head -c 600 $OUT/bench_c2.json
bash tools/profile.sh ${TAG}_c2 --e2e-units 0 --no-frames > /dev/null || exit 1
bash tools/profile.sh ${TAG}_c3 --config c3 --e2e-units 0 --no-frames > /dev/null || exit 1
bash tools/profile.sh ${TAG}_c5 --config c5 --e2e-units 0 --no-frames > /dev/null || exit 1
for c in c3 c5 c4; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c',d['value'],d['kernels'].get('k_resid_ms'),d['roofline']['frac'],(d.get('parity') or {}).get('mismatches'))"
done
