# Parity tests + a short bench + k_resid phase ablation (stop=1,2,0) at 200k units.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
for k in 1 2 0; do
  FLACMI_DEBUG_STOP=$k timeout -k 10 200 python bench.py --units 200000 --steps 5 --warmup 2 --cpu-seconds 0 --no-frames $([ $k -ne 0 ] && echo --no-parity) > gpurun_out/q_$k.json 2>gpurun_out/q_$k.err || { tail gpurun_out/q_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q_$k.json')); print('stop=$k', 'k_resid_ms %.3f' % d['kernels']['k_resid_ms'], 'k_lpc_ms %.3f' % d['kernels']['k_lpc_ms'], 'value %.4g' % d['value'], d.get('parity'))"
done
