# the GPU suite N times in a row (flakiness check); stops at the first failure
N=${1:-2}
mkdir -p gpurun_out/repeat
for i in $(seq 1 $N); do
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:randomly > gpurun_out/repeat/run$i.log 2>&1
  rc=$?; echo "run $i rc=$rc $(tail -1 gpurun_out/repeat/run$i.log)"
  [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " gpurun_out/repeat/run$i.log | head -5; exit 1; }
done
