"""Regenerates the 256-entry table of Julia's table-driven exp (base/special/exp.jl, J_TABLE) from its
defining rule, for include/mp_jlmath.h: entry j packs jU = 2^(j/256) rounded DOWN to Float64 (low 52
mantissa bits) and the top 12 bits of the Float64 jL = RN(2^(j/256) - jU) above bit 44 into bits 52..63
(table_unpack: jU = 0x3FF0<<48 | (e & (2^52-1)), jL = 0x3C00<<48 | (e >> 8)).  Checked against the two
entries quoted in tests/test_jlmath.py (j = 1, 2)."""
import math
import struct
from decimal import Decimal, getcontext

getcontext().prec = 80


def f2u(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def entry(j):
    val = Decimal(2) ** (Decimal(j) / Decimal(256))
    vu = float(val)
    if Decimal(vu) > val:
        vu = math.nextafter(vu, -math.inf)
    vs = float(val - Decimal(vu))
    return (((f2u(vs) >> 44) << 52) | (f2u(vu) & ((1 << 52) - 1))) & 0xFFFFFFFFFFFFFFFF


if __name__ == "__main__":
    ents = [entry(j) for j in range(256)]
    for i in range(0, 256, 4):
        print("    " + ", ".join("0x%016xull" % e for e in ents[i:i + 4]) + ",")
