"""Generate the 2^(k/128) table of csrc/sift_pow2.h (128 pairs of 64-bit
words): word 2k = bits of T_k, word 2k+1 = bits of H_k minus k << 45, where
H_k = RN(2^(k/128)) and T_k = RN(2^(k/128) / H_k - 1), evaluated with 80
decimal digits (Python's float(Decimal) rounds correctly).

usage: python tools/gen_pow2_table.py > table.inc
"""
import struct
from decimal import Decimal, getcontext

getcontext().prec = 80
N = 128


def u64(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def main():
    ln2 = Decimal(2).ln()
    for k in range(N):
        e = (Decimal(k) / N * ln2).exp()
        h = float(e)
        t = float(e / Decimal(h) - 1)
        print(f"    0x{u64(t):016x}ull, 0x{(u64(h) - (k << 45)) % 2**64:016x}ull,")


if __name__ == "__main__":
    main()
