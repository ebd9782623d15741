"""flac_amd — MI355X-native FLAC encode-analysis for turlando/flac-py's encode() API.

The per-block analysis (fixed predictor search, Tukey-windowed autocorrelation,
Levinson-Durbin, LPC quantisation, candidate residuals, subframe choice and Rice
partition search) runs as HIP kernels in ``libflacmi.so`` behind a C-ABI
(``include/flacmi.h``); the encoder entry point, the Subframe/Residual dataclasses
and the bitstream writer keep flac-py's interface (flac/encoder.py, flac/common.py).
"""
__version__ = "0.1.0"
