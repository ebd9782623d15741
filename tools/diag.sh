# Diagnostics on the GPU box: bench with the frame-writer leg, k_resid phase ablation,
# and the list of PMC counters rocprofv3 offers on this device.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --units 200000 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/bench_frames.json 2> gpurun_out/bench_frames.err || { echo bench failed; tail -30 gpurun_out/bench_frames.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_frames.json')); print(d['value'], d['kernels']); print(json.dumps(d['frame_writer']))"
for k in 1 2 3 4 0; do
  FLACMI_DEBUG_STOP=$k timeout -k 10 200 python bench.py --units 200000 --steps 5 --warmup 2 --cpu-seconds 0 --no-parity --no-frames > gpurun_out/abl_$k.json 2>gpurun_out/abl_$k.err || { tail gpurun_out/abl_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abl_$k.json')); print('stop=$k', 'k_resid_ms %.3f' % d['kernels']['k_resid_ms'], 'k_lpc_ms %.3f' % d['kernels']['k_lpc_ms'])"
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
grep -o "SQ_[A-Z_0-9]*" gpurun_out/counters.txt | sort -u | tr '\n' ' ' | head -c 6000
