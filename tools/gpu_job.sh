# scratch GPU job: c2 frame-writer A/B (k_pack32 small window at 7 vs 8 waves a SIMD)
set -o pipefail
OUT=gpurun_out/pack32b
mkdir -p $OUT
for g in 0 8 0 8; do
  FLACMI_PACK_GENERIC=$g timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --e2e-units 0 > $OUT/c2_g$g.json 2> $OUT/c2_g$g.err || { tail -20 $OUT/c2_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_g$g.json'));f=d['frame_writer'];print('g$g',f['ms_per_call'],f['algorithmic_GBs'],f.get('parity'),f['decoder_round_trip']['samples_mismatched'])"
done
