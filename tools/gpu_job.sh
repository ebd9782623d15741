# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5final2; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic_current'], r['library_sha16'], r.get('traffic_library_sha16'))"
for c in c3 c5; do timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 3 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }; python3 -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], r['frac'], r['traffic_current'])"; done
