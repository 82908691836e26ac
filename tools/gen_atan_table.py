"""Table of atan(k/16), k = 0..16, as double-double pairs (hi correctly
rounded, lo = the remainder rounded) for the descriptor's f64 atan2
(sift-project_amd/csrc/sift_math64.h kAtanTab). Evaluated with 60-digit
decimal arithmetic (argument halving + Taylor series)."""
from decimal import Decimal, getcontext

getcontext().prec = 60


def atan(x: Decimal) -> Decimal:
    halvings = 0
    while abs(x) > Decimal("0.1"):  # atan(x) = 2 atan(x / (1 + sqrt(1 + x^2)))
        x = x / (1 + (1 + x * x).sqrt())
        halvings += 1
    s, t, n, x2 = Decimal(0), x, 0, x * x
    while True:
        term = t / (2 * n + 1)
        if abs(term) < Decimal(10) ** -58:
            break
        s += term if n % 2 == 0 else -term
        t *= x2
        n += 1
    return s * (2 ** halvings)


if __name__ == "__main__":
    for k in range(17):
        v = atan(Decimal(k) / 16)
        hi = float(v)
        print(f"{{{hi.hex()}, {float(v - Decimal(hi)).hex()}}},")
