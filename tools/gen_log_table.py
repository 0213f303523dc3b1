"""Regenerates the log_fast and cos2pi_u53 tables of mcmc_clv_model_amd/csrc/fastmath.h (COS_TAB,
LOG_TAB, the ln2 split).

log_fast(x), x > 0 normal:  x = 2^k z with z in [OFF, 2 OFF), OFF = 0x3fe5f800_00000000 (~0.6865),
read off the high word h of x:  t = h - 0x3fe5f800,  k = t >> 20 (arithmetic),  bin i = (t >> 12) & 255,
z = x with high word h - (t & 0xfff00000).  Bin i covers the 4096 high-word values from
0x3fe5f800 + 4096 i; its table entry is (invc, logc) with invc ~ 1 / (bin centre) and
logc = -log(invc) (80-digit decimal, rounded to double).  The bin around 1 (i = 160: z in
[1 - 2^-10, 1 + 2^-9)) has invc = 1, logc = 0, so log x near 1 is log1p(z - 1) with no cancellation.
Then r = fma(z, invc, -1) (|r| <= 2^-9), log x = k ln2 + logc + log1p(r), log1p by its degree-6
Taylor polynomial (truncation |r|^6 / 7 <= 2^-54 / 7 relative).

Usage: python tools/gen_log_table.py   (prints the C source block)
"""
import math
import struct
from decimal import Decimal, getcontext

getcontext().prec = 80
OFF_HI = 0x3FE5F800
N = 256


def from_hi(h):
    return struct.unpack("<d", struct.pack("<Q", (h & 0xFFFFFFFF) << 32))[0]


def table():
    out = []
    for i in range(N):
        lo = from_hi(OFF_HI + i * 4096)
        hi = from_hi(OFF_HI + (i + 1) * 4096)
        if lo <= 1.0 < hi:
            out.append((1.0, 0.0))
            continue
        invc = 1.0 / ((lo + hi) / 2)
        logc = float(-Decimal(invc).ln())
        out.append((invc, logc))
    return out


def ln2_split():
    ln2 = Decimal(2).ln()
    m, e = math.frexp(float(ln2))
    hi = math.ldexp(round(m * 2 ** 42), e - 42)  # 42 bits: k * LN2_HI exact for |k| < 2^11
    return hi, float(ln2 - Decimal(hi))


def cos_table():
    """(cos, sin) of 2 pi j / 1024, j = 0..255 (the first quadrant in 256 steps), 60-digit."""
    from decimal import Decimal as Dd
    getcontext().prec = 60
    pi = Dd("3.14159265358979323846264338327950288419716939937510582097494459")
    out = []
    for j in range(256):
        a = 2 * pi * j / 1024
        # Taylor series at 60 digits (|a| < pi / 2)
        c, s, term, k = Dd(0), Dd(0), Dd(1), 0
        while True:
            if k % 4 == 0:
                c += term
            elif k % 4 == 1:
                s += term
            elif k % 4 == 2:
                c -= term
            else:
                s -= term
            k += 1
            term = term * a / k
            if abs(term) < Dd(10) ** -58:
                break
        out.append((float(c), float(s)))
    return out


def main():
    print("__device__ constexpr double COS_TAB[2 * COS_TAB_N] = {  // (cos, sin) of 2 pi j / 1024")
    rows = [f"{a.hex()}, {b.hex()}," for a, b in cos_table()]
    for j in range(0, 256, 2):
        print("    " + " ".join(rows[j:j + 2]))
    print("};")
    hi, lo = ln2_split()
    print(f"constexpr uint32_t LOG_OFF_HI = 0x{OFF_HI:08x}u;")
    print(f"constexpr double LOG_LN2_HI = {hi.hex()};")
    print(f"constexpr double LOG_LN2_LO = {lo.hex()};")
    print("__device__ constexpr double LOG_TAB[2 * LOG_TAB_N] = {  // (invc, logc) per bin")
    rows = [f"{a.hex()}, {b.hex()}," for a, b in table()]
    for j in range(0, N, 2):
        print("    " + " ".join(rows[j:j + 2]))
    print("};")


if __name__ == "__main__":
    main()
