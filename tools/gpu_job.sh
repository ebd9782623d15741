# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_c4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1; rc=$?; tail -1 $O/pt.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pt.log | head -80; exit 1; }
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --cpu-seconds 0 > $O/b_c4.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_c4.json'));print(d['value'],d['ms_per_step'],d['kernels'])" | cut -c1-400
