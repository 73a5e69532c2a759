#!/usr/bin/env python3
"""Writes a synthetic input file in the reference's stdin format, at any size (SURVEY.md §7.2
bench/gen_synthetic.py): "W1 W2 W3 W4 / Seq1 / N / Seq2 x N", shapes from utils/synthetic.SHAPES.

    python tools/gen_synthetic.py --shape input6 --records 134217728 --out /tmp/big6.txt

Records are written in blocks with vectorised numpy (no per-record Python), so 10^9 letters take seconds.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mpi_openmp_cuda_amd.utils.synthetic import SHAPES  # noqa: E402


def uniform_letters(rng, count):
    """count uniform letters A..Z: random bytes below 234 = 9 * 26 (rejection), reduced mod 26 — several
    times faster than Generator.integers for uint8."""
    parts, have = [], 0
    while have < count:
        raw = np.frombuffer(rng.bytes(int((count - have) * 1.12) + 4096), dtype=np.uint8)
        raw = raw[raw < 234]
        parts.append(raw)
        have += raw.shape[0]
    out = np.concatenate(parts)[:count] if len(parts) > 1 else parts[0][:count].copy()
    out %= 26
    out += ord("A")
    return out


def make_block(rng, n, lo, hi):
    lengths = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    ends = np.cumsum(lengths + 1)  # each record + '\n'
    buf = uniform_letters(rng, int(ends[-1]))
    buf[ends - 1] = ord("\n")
    return buf.tobytes(), int(lengths.sum())


def write_block(f, rng, n, lo, hi):
    buf, letters = make_block(rng, n, lo, hi)
    f.write(buf)
    return letters


def _job_block(args):
    seed, i, n, lo, hi = args
    return make_block(np.random.default_rng([seed, i]), n, lo, hi)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="input6", choices=sorted(SHAPES))
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--block", type=int, default=1 << 22, help="records per write")
    ap.add_argument("--out", required=True)
    ap.add_argument("--jobs", type=int, default=1,
                    help="worker processes generating blocks (block i seeded by (seed, i): a different, equally "
                         "random stream than --jobs 1, the same for every --jobs > 1)")
    a = ap.parse_args()
    s = SHAPES[a.shape]
    rng = np.random.default_rng(a.seed)
    seq1 = "".join(chr(65 + x) for x in rng.integers(0, 26, s.L1))
    letters = 0
    with open(a.out, "wb") as f:
        f.write(f"{' '.join(map(str, s.weights))}\n{seq1}\n{a.records}\n".encode())
        if a.jobs > 1:
            import multiprocessing as mp

            sizes = [min(a.block, a.records - b) for b in range(0, a.records, a.block)]
            with mp.get_context("fork").Pool(a.jobs) as pool:
                for buf, n_letters in pool.imap(_job_block, [(a.seed, i, n, s.l2_min, s.l2_max)
                                                             for i, n in enumerate(sizes)]):
                    f.write(buf)
                    letters += n_letters
        else:
            done = 0
            while done < a.records:
                n = min(a.block, a.records - done)
                letters += write_block(f, rng, n, s.l2_min, s.l2_max)
                done += n
    print(f"{a.out}: {a.records} records, {letters} letters, {os.path.getsize(a.out)} bytes", file=sys.stderr)


if __name__ == "__main__":
    main()
