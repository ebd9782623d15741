# scratch GPU job: frame tests with k_packw as the default writer, then c2/c3/c5 frame legs
set -o pipefail
OUT=gpurun_out/packw_all
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_decode.py tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest.log | head -80; exit 1; }
for spec in c2:0 c2:2 c5:0 c5:2; do
  c=${spec%%:*}; g=${spec##*:}
  FLACMI_PACK_GENERIC=$g timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 --e2e-units 0 > $OUT/${c}_g$g.json 2> $OUT/${c}_g$g.err || { tail -20 $OUT/${c}_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}_g$g.json'));f=d['frame_writer'];print('$c g$g',f['ms_per_call'],f['algorithmic_GBs'],f.get('parity'),f['decoder_round_trip']['samples_mismatched'],f['decoder_round_trip']['frames_with_status'])"
done
