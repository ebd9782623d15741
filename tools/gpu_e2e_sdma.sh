# end-to-end leg with the default copy engines and with HSA_ENABLE_SDMA=0 (blit-kernel copies)
set -o pipefail
OUT=gpurun_out/${1:-e2e_sdma}
mkdir -p $OUT
for v in 1 0; do
  HSA_ENABLE_SDMA=$v timeout -k 10 400 python bench.py --cpu-seconds 0 --no-frames --no-parity --steps 3 > $OUT/bench_sdma$v.json 2> $OUT/bench_sdma$v.err || { tail -20 $OUT/bench_sdma$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_sdma$v.json'));e=d['end_to_end'];print('sdma=$v', d['value'], e['samples_per_s'], e['wall_ms'], e['step_ms'])"
done
