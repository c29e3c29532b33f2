"""Derive spt_powf.h's kExp2Tab: tab[i] = bits(2^(i/32) rounded to double) - (i << 47).

The exp2 table of glibc's powf (__exp2f_data.tab) is defined this way; Decimal at
80 digits and Decimal->float conversion (correctly rounded) give it exactly.
python tools/derive_exp2_table.py   prints the table (tests/test_oracle_kat.py checks it).
"""
import struct
from decimal import Decimal, getcontext


def exp2_table(n=32):
    getcontext().prec = 80
    out = []
    for i in range(n):
        f = float(Decimal(2) ** (Decimal(i) / Decimal(n)))
        out.append(struct.unpack("<Q", struct.pack("<d", f))[0] - (i << (52 - 5)))
    return out


if __name__ == "__main__":
    for i, v in enumerate(exp2_table()):
        print(f"0x{v:016x}ull,", end="\n" if i % 4 == 3 else " ")
