set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "c3 or mf8 or int8 or production" > $O/pt1.log 2>&1; rc=$?; tail -3 $O/pt1.log; [ $rc -eq 0 ] || exit 1
for v in "" "FLACMI_SB=0"; do
  env $v timeout -k 10 200 python bench.py --config c3 --steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0 > $O/c3_${v:-sb}.json 2> $O/c3_${v:-sb}.err || { tail $O/c3_${v:-sb}.err; exit 1; }
  python tools/show_bench.py $O/c3_${v:-sb}.json
done
