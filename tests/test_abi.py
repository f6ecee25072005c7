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


def test_struct_sizes_match_header(tmp_path):
    """ctypes mirrors vs the C compiler's layout of include/mpgpu.h (sizeof + every offsetof)."""
    import subprocess

    structs = {"mp_mppi_params": abi.MPPIParams, "mp_mppi_loop_params": abi.MPPILoopParams,
               "mp_ilqr_params": abi.ILQRParams, "mp_ha_params": abi.HAParams, "mp_track_params": abi.TrackParams}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/mpgpu.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            cf = {"lambda_": "lambda"}.get(fname, fname)  # Python keyword
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {cf}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n") if l)
    for cname, py in structs.items():
        assert int(got[cname]) == abi.ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)

