# GPU suite, the FLACMI_MF8_PERSIST=1 parity subset, then c3 A/B: this build with and without
# FLACMI_MF8_PERSIST vs libflacmi_r04base.so (round-3 tier code); c2 line (tier histograms).
set -o pipefail
TAG=${1:-r04c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
FLACMI_MF8_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lds_guard.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3 or 24bit or int8 or golden or production or lds" > $OUT/pytest_mf8.log 2>&1
rc=$?; echo "pytest (FLACMI_MF8_PERSIST=1) rc=$rc $(tail -1 $OUT/pytest_mf8.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $OUT/pytest_mf8.log | head -60; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0"
for run in default:0 r04base:0 default:1 default:0 r04base:0 default:1; do
  lib=${run%:*}; m=${run#*:}
  if [ $lib = default ]; then L=$PWD/flac-py_amd/libflacmi.so; else L=$PWD/flac-py_amd/libflacmi_$lib.so; fi
  FLACMI_LIB=$L FLACMI_MF8_PERSIST=$m timeout -k 10 200 python bench.py --config c3 $B > $OUT/c3_${lib}_$m.json 2> $OUT/c3_${lib}_$m.err || { tail -20 $OUT/c3_${lib}_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_${lib}_$m.json'));k=d['kernels'];print('c3 $lib MF8_PERSIST=$m', '%.3e'%d['value'], 'lpc %.2f resid %.2f'%(k['k_lpc_ms'],k['k_resid_ms']), (d.get('parity') or {}).get('mismatches'), d['stream_stats']['lpc_tiers'])"
done
timeout -k 10 200 python bench.py --config c2 $B > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c2.json'));k=d['kernels'];print('c2', '%.3e'%d['value'], 'lpc %.2f resid %.2f'%(k['k_lpc_ms'],k['k_resid_ms']), (d.get('parity') or {}).get('mismatches'), d['stream_stats']['lpc_tiers'])"
