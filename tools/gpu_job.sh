# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --config c4 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --e2e-units 0 --no-frames > $O/c4.json 2> $O/tr.err || { tail $O/tr.err; exit 1; }
grep "k_synth\|k_resid_stream\|k_lpc" $O/tr/run_kernel_stats.csv | cut -c1-120
python3 -c "import json; d=json.load(open('$O/c4.json')); print(d['value'], d['ms_per_step'])"
