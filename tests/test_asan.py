"""SURVEY §5 "ASan host build": the CPU-side code under AddressSanitizer + UBSan.

* oracle/asan_check.c drives every oracle entry point over edge shapes (n = 0..16384,
  2..32-bit samples, orders 0..32, every mode, empty Rice ranges, the batch entry point
  with tail units and threads, pow / log2 / Levinson / quantiser on NaN, inf, denormals).
* tests/asan_host_child.py loads a host-ASan build of libflacmi.so (device code unchanged)
  and drives everything that runs without a device: the tables flacmi_create builds, the
  host pow / log2 helpers, and every entry point with NULL arguments.
Both found real defects when added (an out-of-bounds table read for a non-finite
flacmi_host_floor_log2 argument, NULL contexts reaching hipSetDevice)."""
import glob
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan():
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True, timeout=300)
    r = subprocess.run([os.path.join(REPO, "oracle", "_asan", "asan_check")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "no sanitizer report" in r.stdout


def test_host_cabi_under_asan_ubsan():
    csrc = os.path.join(REPO, "flac-py_amd", "csrc")
    if not glob.glob(os.path.join(csrc, "build", "k_*.o")):
        pytest.skip("kernel objects not built (run __graft_entry__.build() first)")
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt:
        pytest.skip("clang ASan runtime not found")
    subprocess.run(["make", "-s", "-C", csrc, "asan"], check=True, timeout=900)
    env = dict(os.environ, LD_PRELOAD=rt[-1], ASAN_OPTIONS="detect_leaks=0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "asan_host_child.py"),
                        os.path.join(csrc, "build", "libflacmi_asan.so")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "no sanitizer report" in r.stdout
