"""Child process of tests/test_asan.py, run with the clang ASan runtime preloaded: loads the
host-ASan build of the C-ABI (flac-py_amd/csrc/build/libflacmi_asan.so) with plain ctypes
(no torch, no device) and drives every entry point that runs without a device: the table
builders behind flacmi_create, the host pow / log2 helpers on edge values, and every
entry point with a NULL context or NULL arguments (each must return an error, not crash)."""
import ctypes as C
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "flac-py_amd"))
import abi  # noqa: E402  (the ctypes mirror; imported standalone, without the package)

lib = C.CDLL(sys.argv[1])
for name, (res, args) in abi.SIGNATURES.items():
    fn = getattr(lib, name)
    fn.restype, fn.argtypes = res, args

assert lib.flacmi_abi_version() == abi.ABI_VERSION
assert lib.flacmi_device_count() == 0, "this check runs where no HIP device is visible"
assert not lib.flacmi_create(0)  # builds the host tables, then finds no device
assert lib.flacmi_last_error()
st = C.c_int32()
for x in (0.0, -0.0, 1.0, -1.0, 1e-310, 1e154, 1.3407807929942596e154, -1.35e154, 1e308, math.inf, -math.inf,
          math.nan, 0.5, 2.0, 5e-324, 1 - 2 ** -53):
    lib.flacmi_host_pypow2(x, C.byref(st))
    lib.flacmi_host_floor_log2(x)
for k in range(-1074, 1024, 7):
    lib.flacmi_host_floor_log2(math.ldexp(1.0, k))
    lib.flacmi_host_floor_log2(math.ldexp(1.0, k) * (1 - 2 ** -53))

skip = {"flacmi_abi_version", "flacmi_last_error", "flacmi_device_count", "flacmi_create",
        "flacmi_host_pypow2", "flacmi_host_floor_log2", "flacmi_comm_available"}
calls = 0
for name, (res, args) in abi.SIGNATURES.items():
    if name in skip:
        continue
    fn = getattr(lib, name)
    r = fn(*[None if a is not C.c_int and a is not C.c_int32 and a is not C.c_int64 and a is not C.c_size_t
             and a is not C.c_uint64 and a is not C.c_double else 0 for a in args])
    calls += 1
    if name in ("flacmi_host_free", "flacmi_comm_destroy"):
        assert r == 0  # freeing / destroying NULL is a no-op
    elif res is C.c_int:
        assert r != 0, f"{name} accepted a NULL context"
    elif res is C.c_void_p:
        assert not r, f"{name} returned memory for a NULL context"
print(f"asan host: tables, pow/log2 helpers and {calls} entry points with NULL arguments, no sanitizer report")
