"""libflacmi.so loads, reports its ABI version and exports every symbol include/flacmi.h
declares (CPU-only: no compute call needs a GPU here)."""
import ctypes
import os
import re

from flac_amd import abi
from flac_amd._lib import LIB_PATH, load

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "flacmi.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(flacmi_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_abi_version():
    lib = load()
    assert lib.flacmi_abi_version() == abi.ABI_VERSION


def test_every_declared_symbol_is_exported_and_typed():
    lib = ctypes.CDLL(LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), f"{name} declared in include/flacmi.h but not exported"
        assert name in abi.SIGNATURES, f"{name} missing from flac_amd.abi.SIGNATURES"


def test_struct_layouts_match_header(tmp_path):
    """Every field offset of the ctypes mirror equals the C compiler's offsetof()."""
    import subprocess
    structs = {"flacmi_params": abi.Params, "flacmi_batch": abi.Batch,
               "flacmi_unit_meta": abi.UnitMeta, "flacmi_outputs": abi.Outputs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, f"{cname}.{f}"
    assert abi.META_DTYPE.itemsize == ctypes.sizeof(abi.UnitMeta)


def test_create_without_device_fails_loudly():
    lib = load()
    if lib.flacmi_device_count() > 0:
        return
    assert not lib.flacmi_create(0)
    assert b"device" in lib.flacmi_last_error()
