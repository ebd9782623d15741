# scratch GPU job: frame-writer tests, then c2 frame-writer A/B (k_pack32 window / occupancy)
set -o pipefail
OUT=gpurun_out/pack32a
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest.log | head -80; exit 1; }
for g in 0 7 0 7; do
  FLACMI_PACK_GENERIC=$g timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --e2e-units 0 > $OUT/c2_g$g.json 2> $OUT/c2_g$g.err || { tail -20 $OUT/c2_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_g$g.json'));f=d['frame_writer'];print('g$g',f['ms_per_call'],f['algorithmic_GBs'],f.get('parity'),f['decoder_round_trip']['samples_mismatched'])"
done
