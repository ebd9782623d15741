# parity tests (LPC-related subset) + one full-size config-2 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-frames > gpurun_out/b1.json 2>gpurun_out/b1.err || { tail gpurun_out/b1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b1.json')); k=d['kernels']; print('ms/step %.3f' % d['ms_per_step'], 'lpc %.3f resid %.3f call %.3f' % (k['k_lpc_ms'], k['k_resid_ms'], k['call_ms']), 'value %.4g' % d['value'], 'frac %.3f' % d['roofline']['frac'], d['parity'])"
