# scratch GPU job: frame-writer tests (k_packw edge cases)
set -o pipefail
OUT=gpurun_out/packw5
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest.log | head -80; exit 1; }
