# scratch GPU job: k_packw 4 KB vs 2 KB ring on c2 and c3 frames
set -o pipefail
OUT=gpurun_out/packw_r2k
mkdir -p $OUT
for spec in c2:0 c2:9 c3:0 c3:9 c2:0 c2:9 c3:0 c3:9; do
  c=${spec%%:*}; g=${spec##*:}
  FLACMI_PACK_GENERIC=$g timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 --e2e-units 0 > $OUT/${c}_g$g.json 2> $OUT/${c}_g$g.err || { tail -20 $OUT/${c}_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}_g$g.json'));f=d['frame_writer'];print('$c g$g',f['ms_per_call'],f['algorithmic_GBs'],f.get('parity'),f['decoder_round_trip']['samples_mismatched'],f['decoder_round_trip']['frames_with_status'])"
done
