# scratch GPU job: the whole GPU suite and smoke on the committed tree
set -o pipefail
OUT=gpurun_out/final_suite
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $OUT/pytest_gpu.log | head -60; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
