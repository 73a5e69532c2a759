"""Exhaustive checks of the multiply-by-reciprocal constants the device decoders use
(csrc/src/hip/swipe_impl.hpp: decode_p33_field, record_words_p33, len6_digit / lane_length6). numpy,
CPU only.

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
    # record_words_p33: q0 / 7 = (q0 * 9363) >> 16 for every record start q0 <= 6 + 63 * 64 of a tile
    check_range(0, 13110, lambda v: (v * U64(9363)) >> U64(16), lambda v: v // U64(7))
    assert (13110 * 9363) >> 16 != 13110 // 7
    # base-6 length digits (lane_length6): octet v < 2^21, digit j = (v / 6^j) - 6 (v / 6^(j+1)), each
    # quotient trunc((v + 0.5) * fl(1 / 6^i)) in f32 (round-to-nearest product), i = 0..8
    v = np.arange(1 << 21, dtype=np.uint32)
    fv = v.astype(np.float32) + np.float32(0.5)
    for i in range(9):
        q = np.trunc(fv * np.float32(1.0 / 6 ** i)).astype(np.int64)
        assert (q == v // 6 ** i).all(), i
    # the lane's octet position: u / 3 = (u * 11) >> 5 for u = (8 t) % 3 + lane / 8 <= 9
    assert all(((u * 11) >> 5) == u // 3 for u in range(10))
    print("ok")


if __name__ == "__main__":
    main()
