"""Exhaustive checks of the multiply-by-reciprocal constants the device decoders use
(csrc/src/hip/swipe_impl.hpp: decode_p33_field, len6_digit / lane_length6). numpy, CPU only.

    python tools/p33_magic_check.py
"""
import numpy as np

U64 = np.uint64


def check_range(lo, hi, fn, want, chunk=1 << 26):
    for s in range(lo, hi, chunk):
        v = np.arange(s, min(s + chunk, hi), dtype=U64)
        assert (fn(v) == want(v)).all(), (fn, s)


def main():
    n = 26 ** 7  # a P33 field's value range
    m = -(-(1 << 46) // 28561)
    assert m == 2463805336
    # A = umulhi(x >> 4, m) >> 14 == (x >> 4) // 13^4 for every x >> 4 of a field
    check_range(0, (n >> 4) + 1, lambda v: ((v * U64(m)) >> U64(32)) >> U64(14), lambda v: v // U64(28561))
    m676 = -(-(1 << 32) // 676)
    assert m676 == 6353502 and m676 < (1 << 24)  # a v_mul_hi_u32_u24 operand
    check_range(0, 1 << 19, lambda v: (v * U64(m676)) >> U64(32), lambda v: v // U64(676))
    check_range(0, 676, lambda v: (v * U64(2521)) >> U64(16), lambda v: v // U64(26))
    # base-6 length digits: octet v < 2^21, digit j = (v / 6^j) % 6
    ms = [0, 2863311531, 3817748708, 2545165806, 3393554407, 2262369605, 3016492806, 4021990408]
    shs = [0, 2, 5, 7, 10, 12, 15, 18]
    for j in range(1, 8):
        assert ms[j] == -(-(1 << (32 + shs[j])) // 6 ** j) and ms[j] < (1 << 32)
        check_range(0, 1 << 21, lambda v, j=j: ((v * U64(ms[j])) >> U64(32)) >> U64(shs[j]),
                    lambda v, j=j: v // U64(6 ** j))
    check_range(0, 1 << 21, lambda v: (v * U64(715827883)) >> U64(32), lambda v: v // U64(6))
    print("ok")


if __name__ == "__main__":
    main()
