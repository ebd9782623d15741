"""FLAC data model with the field names and values of flac/common.py.

Only what the encoder boundary and the frame writer need: the Subframe*/Residual value
types the analysis fills (flac/common.py:276-420) and the header enums/encodings the
writer uses (:24-271).  Equality of these frozen dataclasses is per class, exactly as in
the reference, so results compare field by field.
"""
from dataclasses import dataclass
from enum import Enum
from typing import Optional, Sequence

MAGIC = b"fLaC"
FRAME_SYNC_CODE = 0b111111111111100
CRC8_POLYNOMIAL = 0x107   # x^8 + x^2 + x + 1
CRC16_POLYNOMIAL = 0x18005  # x^16 + x^15 + x^2 + 1

# order k: the k-th difference predictor
FIXED_PREDICTOR_COEFFICIENTS = ((), (1,), (2, -1), (3, -3, 1), (4, -6, 4, -1))


class MetadataBlockType(Enum):
    Streaminfo = 0
    Padding = 1
    Application = 2
    Seektable = 3
    VorbisComment = 4
    Cuesheet = 5
    Picture = 6


@dataclass(frozen=True)
class MetadataBlockHeader:
    last: bool
    type: MetadataBlockType
    length: int


@dataclass(frozen=True)
class Streaminfo:
    min_block_size: int
    max_block_size: int
    min_frame_size: int
    max_frame_size: int
    sample_rate: int
    channels: int
    sample_size: int
    samples: int
    md5: bytes


class BlockingStrategy(Enum):
    Fixed = 0
    Variable = 1


@dataclass(frozen=True)
class BlockSizeValue:
    size: int


@dataclass(frozen=True)
class BlockSizeUncommon8:
    pass


@dataclass(frozen=True)
class BlockSizeUncommon16:
    pass


BlockSize = BlockSizeValue | BlockSizeUncommon8 | BlockSizeUncommon16

# frame-header block-size codes: 192, 144*2^k (k=2..5), 2^k (k=8..15)
BLOCK_SIZE_ENCODING = {192: 0b0001}
BLOCK_SIZE_ENCODING.update({144 << k: 0b0010 + k - 2 for k in range(2, 6)})
BLOCK_SIZE_ENCODING.update({1 << k: 0b1000 + k - 8 for k in range(8, 16)})


class SampleRateFromStreaminfo:
    pass


class SampleRateValue(Enum):
    V_88_2_kHz = 88_200
    V_176_4_kHz = 176_400
    V_192_kHz = 192_000
    V_8_kHz = 8_000
    V_16_kHz = 16_000
    V_22_05_kHz = 22_050
    V_24_kHz = 24_000
    V_32_kHz = 32_000
    V_44_1_kHz = 44_100
    V_48_kHz = 48_000
    V_96_kHz = 96_000

    @classmethod
    def values(cls):
        return {m.value for m in cls}


class SampleRateUncommon8:
    pass


class SampleRateUncommon16:
    pass


class SampleRateUncommon16_10:
    pass


SampleRate = (SampleRateFromStreaminfo | SampleRateValue | SampleRateUncommon8
              | SampleRateUncommon16 | SampleRateUncommon16_10)

# codes 0b0001..0b1011 in declaration order, then 96 kHz at 0b1100
SAMPLE_RATE_VALUE_ENCODING = {m: i + 1 for i, m in enumerate(list(SampleRateValue)[:10])}
SAMPLE_RATE_VALUE_ENCODING[SampleRateValue.V_96_kHz] = 0b1100


class Channels(Enum):
    M = 1
    L_R = 2
    L_R_C = 3
    FL_FR_BL_BR = 4
    FL_FR_FC_BL_BR = 5
    FL_FR_FC_LFE_BL_BR = 6
    FL_FR_FC_LFE_BC_SL_SR = 7
    FL_FR_FC_LFE_BL_BR_SL_SR = 8
    L_S = 9
    S_R = 10
    M_S = 11

    @property
    def count(self) -> int:
        return 2 if self.value > 8 else self.value


CHANNELS_ENCODING = {c: i for i, c in enumerate(Channels)}


@dataclass(frozen=True)
class SampleSizeFromStreaminfo:
    pass


class SampleSizeValue(Enum):
    V_8 = 8
    V_12 = 12
    V_16 = 16
    V_20 = 20
    V_24 = 24
    V_32 = 32


SampleSize = SampleSizeFromStreaminfo | SampleSizeValue

SAMPLE_SIZE_ENCODING = dict(zip(SampleSizeValue, (0b001, 0b010, 0b100, 0b101, 0b110, 0b111)))


@dataclass(frozen=True)
class FrameHeader:
    blocking_strategy: BlockingStrategy
    block_size: int
    sample_rate: Optional[int]
    channels: Channels
    sample_size: Optional[int]
    coded_number: int
    crc: Optional[int] = None


# ------------------------------------------------------------------ subframes

@dataclass(frozen=True)
class SubframeTypeConstant:
    pass


@dataclass(frozen=True)
class SubframeTypeVerbatim:
    pass


@dataclass(frozen=True)
class SubframeTypeFixed:
    order: int


@dataclass(frozen=True)
class SubframeTypeLPC:
    order: int


SubframeType = SubframeTypeConstant | SubframeTypeVerbatim | SubframeTypeFixed | SubframeTypeLPC


@dataclass(frozen=True)
class SubframeHeader:
    type_: SubframeType
    wasted_bits: int


@dataclass(frozen=True)
class SubframeConstant:
    sample: int
    block_size: int

    def __repr__(self):
        return "SubframeConstant()"


@dataclass(frozen=True)
class SubframeVerbatim:
    samples: list

    def __repr__(self):
        return "SubframeVerbatim()"


@dataclass(frozen=True)
class SubframeFixed:
    warmup: list
    residual: list

    @property
    def order(self) -> int:
        return len(self.warmup)

    def __repr__(self):
        return f"SubframeFixed(order={self.order})"


@dataclass(frozen=True)
class SubframeLPC:
    warmup: list
    precision: int
    shift: int
    coefficients: list
    residual: list

    @property
    def order(self) -> int:
        return len(self.warmup)

    def __repr__(self):
        return (f"SubframeLPC(order={self.order}, precision={self.precision}, "
                f"shift={self.shift}, coefficients={self.coefficients})")


Subframe = SubframeConstant | SubframeVerbatim | SubframeFixed | SubframeLPC


@dataclass(frozen=True)
class Frame:
    header: FrameHeader
    subframes: list
    crc: int


@dataclass(frozen=True)
class RicePartition:
    parameter: int
    residual: list  # zig-zag encoded

    def __repr__(self):
        return f"RicePartition(parameter={self.parameter}, samples_count={len(self.residual)})"


@dataclass(frozen=True)
class EscapedPartition:
    residual: list

    def __repr__(self):
        return f"EscapedPartition(samples_count={len(self.residual)})"


ResidualPartition = RicePartition | EscapedPartition


class RiceCodingMethod(Enum):
    Rice4Bit = 4
    Rice5Bit = 5


@dataclass(frozen=True)
class Residual:
    coding_method: RiceCodingMethod
    partitions: Sequence

    @property
    def partition_order(self) -> int:
        return len(self.partitions).bit_length() - 1

    def __repr__(self):
        return (f"Residual(coding_method={self.coding_method}, "
                f"partition_order={self.partition_order}, partitions={self.partitions})")
