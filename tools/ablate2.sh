# k_resid ablation for both candidate-sum paths: FLACMI_DEBUG_STOP=1..4,0 x FLACMI_NO_MFMA=0/1
set -o pipefail
mkdir -p gpurun_out
for m in 0 1; do
for k in 1 2 3 4 0; do
  FLACMI_NO_MFMA=$m FLACMI_DEBUG_STOP=$k timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-parity "$@" > gpurun_out/abl_$m$k.json 2>gpurun_out/abl_$m$k.err || { tail gpurun_out/abl_$m$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abl_$m$k.json')); print('nomfma=$m stop=$k', 'k_resid_ms %.2f' % d['kernels']['k_resid_ms'])"
done
done
