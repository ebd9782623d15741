# GPU suite, then c3 A/B on one box: the sign-correlation bound (default) vs the partial-sum
# tiers alone (FLACMI_NO_SIGNBOUND=1), with the tier histogram.  Usage: bash tools/gpu_r04o.sh <tag>
set -o pipefail
TAG=${1:-r04o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0"
for v in 0 1 0 1; do
  FLACMI_NO_SIGNBOUND=$v timeout -k 10 200 python bench.py --config c3 $B > $OUT/c3_nsb$v.json 2> $OUT/c3_nsb$v.err || { tail -20 $OUT/c3_nsb$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_nsb$v.json'));k=d['kernels'];print('c3 NO_SIGNBOUND=$v', '%.4e'%d['value'], 'lpc %.3f resid %.3f call %.3f'%(k['k_lpc_ms'],k['k_resid_ms'],k['call_ms']), (d.get('parity') or {}).get('mismatches'), d['stream_stats'].get('lpc_tiers'))"
done
