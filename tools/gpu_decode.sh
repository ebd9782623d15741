# decoder tests, then the c2 frame-writer leg (frames + decoder round trip)
set -o pipefail
OUT=gpurun_out/${1:-dec}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head; exit 1; }
timeout -k 10 400 python bench.py --cpu-seconds 0 --e2e-units 0 --steps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));f=d['frame_writer'];print('pack ms',f['ms_per_call'],'decode', json.dumps(f['decoder_round_trip'])[:300])"
