#!/usr/bin/env python3
"""Constants of the shared Julia-Base libm restatement (gppupildemodulation.jl_amd/csrc/
gpd_jlmath.h), derived from exact integer arithmetic rather than copied:

  * INV_2PI: 1/(2π) as 19 big-endian 64-bit words (Julia's table in base/special/rem_pio2.jl,
    used by the Payne–Hanek reduction for |x| ≥ 2^20·π/2), from π by Machin's formula
    π = 16 atan(1/5) − 4 atan(1/239) in fixed point with guard bits;
  * the hypot thresholds sqrt(eps/2) and sqrt(floatmax/2) (base/math.jl), correctly rounded.

Run it to print the table; tests/test_jlmath.py compares it with the header."""
import math
import sys

WORDS = 19


def pi_fixed(bits: int) -> int:
    """floor(π·2^bits) (to within one unit), Machin's formula with 64 guard bits."""
    guard = 64
    one = 1 << (bits + guard)

    def atan_inv(x: int) -> int:  # atan(1/x)·one
        total = term = one // x
        x2 = x * x
        n, sign = 1, -1
        while term:
            term //= x2
            total += sign * (term // (2 * n + 1))
            sign, n = -sign, n + 1
        return total

    return (16 * atan_inv(5) - 4 * atan_inv(239)) >> guard


def inv2pi_words(words: int = WORDS) -> list[int]:
    """The first `words` 64-bit words of the binary expansion of 1/(2π)."""
    width = 64 * words
    extra = 128
    p = pi_fixed(width + extra)  # π·2^(width+extra)
    q = (1 << (2 * width + 2 * extra)) // (2 * p)  # 2^(width+extra)/(2π)
    q >>= extra
    return [(q >> (64 * (words - 1 - i))) & ((1 << 64) - 1) for i in range(words)]


def hypot_thresholds() -> dict:
    return {"sqrt(eps/2)": math.sqrt(2.0 ** -53).hex(),
            "sqrt(floatmax/2)": math.sqrt(sys.float_info.max / 2).hex()}


if __name__ == "__main__":
    ws = inv2pi_words()  # the JLM_INV2PI_WORDS table of csrc/gpd_jlmath.h
    print(",\n".join(", ".join(f"0x{w:016x}ull" for w in ws[i:i + 3]) for i in range(0, len(ws), 3)))
    print(hypot_thresholds())
