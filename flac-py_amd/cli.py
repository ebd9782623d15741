"""Command line with flac/__main__.py's `encode` action (its arguments, defaults and
output bytes), on the device path: streamed PCM ingest (ingest.iter_wav_pcm, the
reference reader's byte grouping unless --correct-reader), device analysis and device
frame writer through the streaming pipeline (encoder.encode_wav); --devices spreads the
batches over several GPUs.

    python -m flac_amd encode infile.wav outfile.flac [-b N] [-l N] [-q N] [-r [M,]N]
                                                       [--correct-reader] [--fixed-only]
                                                       [--device N | --devices N,M,...]

The reference's `decode` action (a WAV writer over its host decoder) is not part of this
build; the device decoder (flacmi_decode_frames_device) is a frame verifier.
"""
import argparse
import sys
from pathlib import Path
from timeit import default_timer as timer

from .utils import argparse_range

DEFAULT_BLOCK_SIZE = 4608
DEFAULT_MAX_LPC_ORDER = 12
DEFAULT_QLP_COEFF_PRECISION = 5
DEFAULT_RICE_PARTITION_ORDER = "5"


def make_argument_parser():
    parser = argparse.ArgumentParser(prog="flac_amd", formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    action = parser.add_subparsers(title="action", dest="action", required=True)
    enc = action.add_parser("encode", formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    enc.add_argument("infile", type=Path, metavar="infile.wav")
    enc.add_argument("outfile", type=Path, metavar="outfile.flac")
    enc.add_argument("-b", "--block-size", type=int, default=DEFAULT_BLOCK_SIZE, metavar="N")
    enc.add_argument("-l", "--max-lpc-order", type=int, default=DEFAULT_MAX_LPC_ORDER, metavar="N")
    enc.add_argument("-q", "--qlp-coeff-precision", type=int, default=DEFAULT_QLP_COEFF_PRECISION, metavar="N")
    enc.add_argument("-r", "--rice-partition-order", type=argparse_range, default=DEFAULT_RICE_PARTITION_ORDER,
                     metavar="[M,]N")
    enc.add_argument("--correct-reader", action="store_true",
                     help="read sampwidth-byte samples (the reference groups frame bytes by channel count)")
    enc.add_argument("--fixed-only", action="store_true", help="fixed predictors only (BASELINE config 5)")
    enc.add_argument("--device", type=int, default=0)
    enc.add_argument("--devices", type=lambda v: [int(x) for x in v.split(",")], default=None, metavar="N,M,...",
                     help="encode on these devices, batches round-robin (frames in block order)")
    return parser


def cmd_encode(args) -> None:
    from .encoder import EncoderParameters, encode_wav
    parameters = EncoderParameters(block_size=args.block_size, lpc_order=range(args.max_lpc_order + 1),
                                   qlp_precision=args.qlp_coeff_precision,
                                   rice_partition_order=args.rice_partition_order)
    t0 = timer()
    with args.outfile.open("wb") as f:
        for bs in encode_wav(args.infile, parameters, quirk=not args.correct_reader, device=args.device,
                             devices=args.devices, fixed_only=args.fixed_only):
            f.write(bs)
    print(f"Encoding completed in {timer() - t0:.6g} seconds")


def main(argv=None) -> int:
    args = make_argument_parser().parse_args(argv)
    if args.action == "encode":
        cmd_encode(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
