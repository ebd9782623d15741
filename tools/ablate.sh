# k_resid phase ablation: bench timing with the kernel truncated after each phase.
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3 4 0; do
  FLACMI_DEBUG_STOP=$k timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-parity "$@" > gpurun_out/abl_$k.json 2>gpurun_out/abl_$k.err || { tail gpurun_out/abl_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abl_$k.json')); print('stop=$k', 'k_resid_ms %.2f' % d['kernels']['k_resid_ms'], 'k_lpc_ms %.2f' % d['kernels']['k_lpc_ms'])"
done
