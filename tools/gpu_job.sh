# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -60; exit 1; }
for g in 2048 8192 16384; do
  FLACMI_LIST_GRID=$g timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0 > $O/c2_g$g.json 2> $O/err || { tail $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_g$g.json'));k=d['kernels'];print('grid $g', '%.4e'%d['value'], 'lpc %.3f resid %.3f call %.3f'%(k['k_lpc_ms'],k['k_resid_ms'],k['call_ms']))"
done
