# Round-4 A/B on one box: c3 k_resid default vs FLACMI_MF8_1024=1 (parity tests of the
# 24-bit paths under it first), c2 k_lpc tile vs FLACMI_LPC_TILE=0.  Usage: bash tools/gpu_ab_r04.sh <tag>
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
FLACMI_MF8_1024=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lds_guard.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3 or 24bit or int8 or golden or production or lds" > $OUT/pytest_mf8.log 2>&1
rc=$?; echo "pytest (FLACMI_MF8_1024=1) rc=$rc $(tail -1 $OUT/pytest_mf8.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $OUT/pytest_mf8.log | head -60; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0"
for v in 0 1 0 1; do
  FLACMI_MF8_1024=$v timeout -k 10 200 python bench.py --config c3 $B > $OUT/c3_mf8_$v.json 2> $OUT/c3_mf8_$v.err || { tail -20 $OUT/c3_mf8_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_mf8_$v.json'));k=d['kernels'];print('c3 MF8_1024=$v', '%.3e'%d['value'], 'lpc %.2f resid %.2f'%(k['k_lpc_ms'],k['k_resid_ms']), (d.get('parity') or {}).get('mismatches'), d['stream_stats']['lpc_pruned'])"
done
for v in 0 1 0 1; do
  FLACMI_LPC_TILE=$v timeout -k 10 200 python bench.py --config c2 $B > $OUT/c2_tile_$v.json 2> $OUT/c2_tile_$v.err || { tail -20 $OUT/c2_tile_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_tile_$v.json'));k=d['kernels'];print('c2 LPC_TILE=$v', '%.3e'%d['value'], 'lpc %.2f resid %.2f'%(k['k_lpc_ms'],k['k_resid_ms']), (d.get('parity') or {}).get('mismatches'))"
done
