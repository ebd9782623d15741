# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lds_guard.py -x -q --timeout 120 --timeout-method thread -k "c3 or mf8 or int8 or production or every_order or golden or lds" > $O/pt.log 2>&1; rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -60; exit 1; }
STOPS="1 2 4 5 6 7 0" bash tools/ablate.sh r5k/abl --config c3
