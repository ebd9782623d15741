# scratch GPU job: c3 frame-writer A/B (k_packw 256 vs 128 vs 64 threads)
set -o pipefail
OUT=gpurun_out/packw64
mkdir -p $OUT
for g in 0 6 8 0 6 8; do
  FLACMI_PACK_GENERIC=$g timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --cpu-seconds 0 --e2e-units 0 > $OUT/c3_g$g.json 2> $OUT/c3_g$g.err || { tail -20 $OUT/c3_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_g$g.json'));f=d['frame_writer'];print('g$g',f['ms_per_call'],f['algorithmic_GBs'],f.get('parity'),f['decoder_round_trip']['samples_mismatched'],f['decoder_round_trip']['frames_with_status'])"
done
