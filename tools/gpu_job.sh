# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g2; mkdir -p $O
timeout -k 10 400 python bench.py --config c4 --open 0 --steps 3 --warmup 1 --cpu-seconds 3 > $O/bench_c4_o0.json 2> $O/bench_c4_o0.err || { tail -20 $O/bench_c4_o0.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c4_o0.json'));print('c4',d['value'],d['kernels'].get('k_resid_ms'),d['roofline']['frac'],(d.get('parity') or {}).get('mismatches'),d['stream_stats']['lpc_tiers'])"
