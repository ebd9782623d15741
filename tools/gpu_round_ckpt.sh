# Round checkpoint: GPU suite, smoke, default bench line, rocprof trace + FETCH/WRITE for c2, c3,
# c5 and the open-mix lines (--open 5: LPC near-ties no bound decides), bench lines for the
# other configs, FLACMI_NO_PRUNE=1 lines (every candidate exact) and the non-BASELINE b4096.
# Usage: bash tools/gpu_round_ckpt.sh <tag> [quick|part1|part2]
#   quick: no GPU suite, no smoke; part1: suite, smoke, default line, frame-writer/decoder trace,
#   c2/c3/c5 profiles; part2: the open-mix profiles and the other bench lines (two gpurun calls)
set -o pipefail
TAG=${1:-ckpt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
PART=${2:-all}
if [ "$PART" != part2 ]; then
if [ "$PART" != quick ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
  [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $OUT/pytest_gpu.log | head -60; exit 1; }
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python tools/show_bench.py $OUT/bench_c2.json 2>/dev/null || head -c 600 $OUT/bench_c2.json
bash tools/profile.sh ${TAG}_c2 --e2e-units 0 --no-frames > /dev/null || exit 1
bash tools/profile.sh ${TAG}_c3 --config c3 --e2e-units 0 --no-frames > /dev/null || exit 1
bash tools/profile.sh ${TAG}_c5 --config c5 --e2e-units 0 --no-frames > /dev/null || exit 1
# the frame writer and the decoder round trip (k_pack32, k_decode_fx, k_decode) per kernel
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/frames_trace -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-parity > $OUT/bench_frames_trace.json 2> $OUT/frames_trace.err || { tail $OUT/frames_trace.err; exit 1; }
fi
[ "$PART" = part1 ] && exit 0
bash tools/profile.sh ${TAG}_c2_open5 --open 5 --e2e-units 0 --no-frames > /dev/null || exit 1
bash tools/profile.sh ${TAG}_c3_open5 --config c3 --open 5 --e2e-units 0 --no-frames > /dev/null || exit 1
for spec in c3:0 c5:0 c4:0 b4096:0 c2:5 c3:5 c2:8 c3:8; do
  c=${spec%%:*}; k=${spec##*:}
  timeout -k 10 400 python bench.py --config $c --open $k --steps 3 --warmup 1 --cpu-seconds 3 > $OUT/bench_${c}_o$k.json 2> $OUT/bench_${c}_o$k.err || { tail -20 $OUT/bench_${c}_o$k.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${c}_o$k.json'));print('$c o$k',d['value'],d['kernels'].get('k_resid_ms'),d['roofline']['frac'],(d.get('parity') or {}).get('mismatches'),d['stream_stats']['lpc_tiers'])"
done
for spec in c2:0 c3:0 c2:5 c3:5; do
  c=${spec%%:*}; k=${spec##*:}
  FLACMI_NO_PRUNE=1 timeout -k 10 400 python bench.py --config $c --open $k --steps 3 --warmup 1 --cpu-seconds 0 --e2e-units 0 --no-frames > $OUT/bench_${c}_o${k}_noprune.json 2> $OUT/bench_${c}_o${k}_noprune.err || { tail -20 $OUT/bench_${c}_o${k}_noprune.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${c}_o${k}_noprune.json'));print('$c o$k noprune',d['value'],d['kernels'].get('k_resid_ms'),d['roofline']['frac'],(d.get('parity') or {}).get('mismatches'))"
done
