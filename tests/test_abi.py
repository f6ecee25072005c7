"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU calls)."""
import os
import re

from motionplanning_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "mpgpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mp_[a-z0-9_]+)\s*\(", txt)))


def test_all_declared_symbols_exported():
    lib = abi.load_library()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(abi.SIGNATURES), set(syms) ^ set(abi.SIGNATURES)


def test_version_and_no_device_error():
    lib = abi.load_library()
    assert lib.mp_version().decode().startswith("0.1")


def test_struct_sizes_match_header():
    # natural alignment of the POD structs as laid out by the C compiler
    assert abi.ctypes.sizeof(abi.MPPIParams) == 4 * 4 + 8 * 2 + 8 * 4 + 8 * 14 + 8 * 4 + 8 * 2 + 4 * 2 + 8 * 4 + 4 * 2 + 8 * 2
    assert abi.ctypes.sizeof(abi.ILQRParams) == 4 * 2 + 8 * 4 + 4 * 2
