# pruned vs unpruned stream kernel on config 2, with phase stops (timing only)
set -o pipefail
OUT=gpurun_out/${1:-pab}
mkdir -p $OUT
for np in 0 1; do
  for k in 2 3 0; do
    FLACMI_NO_PRUNE=$np FLACMI_DEBUG_STOP=$k timeout -k 10 200 python bench.py --cpu-seconds 0 --no-frames --no-parity --e2e-units 0 --steps 10 > $OUT/np${np}_s$k.json 2> $OUT/np${np}_s$k.err || { tail -5 $OUT/np${np}_s$k.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/np${np}_s$k.json'));print('no_prune=$np stop=$k k_resid %.3f' % d['kernels']['k_resid_ms'])"
  done
done
