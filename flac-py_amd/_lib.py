"""Loader for libflacmi.so (the HIP kernels behind include/flacmi.h).

There is no fallback: if the library is missing or no HIP device is present the
calls fail loudly with FlacmiError.
"""
import ctypes as C
import os

from . import abi

LIB_PATH = os.environ.get("FLACMI_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                     "libflacmi.so"))
_lib = None


class FlacmiError(RuntimeError):
    """A libflacmi.so API call failed (argument, HIP runtime or unsupported shape); `code`
    is the FLACMI_E_* return value when there is one."""
    code = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FlacmiError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (or make -C flac-py_amd/csrc)")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 and binds
        # device buffers/streams to it.  Loading torch first makes libflacmi.so resolve the
        # same soname to that runtime; loaded the other way round torch finds no device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in abi.SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.flacmi_abi_version()
        if v != abi.ABI_VERSION:
            raise FlacmiError(f"libflacmi ABI {v} != {abi.ABI_VERSION}")
        _lib = lib
    return _lib


def check(rc: int, what: str = "flacmi") -> None:
    if rc != 0:
        msg = load().flacmi_last_error().decode(errors="replace")
        err = FlacmiError(f"{what} failed ({rc}): {msg}")
        err.code = rc
        raise err


def last_error() -> str:
    return load().flacmi_last_error().decode(errors="replace")
