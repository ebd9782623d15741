# bench at the full config-2 size with k_lpc/k_resid overlap off and on (FLACMI_OVERLAP chunks)
set -o pipefail
mkdir -p gpurun_out
for k in 0 2 4 8; do
  FLACMI_OVERLAP=$k timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0 > gpurun_out/ov_$k.json 2>gpurun_out/ov_$k.err || { tail gpurun_out/ov_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ov_$k.json')); k=d['kernels']; print('overlap=$k', 'ms/step %.3f' % d['ms_per_step'], 'lpc %.3f resid %.3f call %.3f' % (k['k_lpc_ms'], k['k_resid_ms'], k['call_ms']), 'value %.4g' % d['value'], d['parity']['mismatches'])"
done
