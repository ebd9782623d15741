# Quick GPU cycle: parity tests, then the default bench (c2), then optional extra args.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 600 python bench.py --cpu-seconds 2 "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('value %.4g samples/s  ms/step %.2f' % (d['value'], d['ms_per_step']))
print('kernels', {k: round(v,3) for k,v in d['kernels'].items()})
print('roofline', d['roofline']['kernel'], round(d['roofline']['frac'],4), 'parity', d['parity'])"
