#!/usr/bin/env python3
"""Sums rocprofv3 --pmc counter CSVs per kernel name (prefix before '<'), over every dispatch, and prints
one JSON line per kernel with the counters and derived ratios (VALU instructions per wave cycle, waits).

    python tools/pmc_summary.py [--tag PASS] gpurun_out/pmc_r4_0/p1 gpurun_out/pmc_r4_0/p2
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                key = name.split("(")[0]
                ctr = row.get("Counter_Name")
                try:
                    val = float(row.get("Counter_Value", "0"))
                except ValueError:
                    continue
                tot[key][ctr] += val
                disp[key].add(row.get("Dispatch_Id"))
    return tot, disp


def main(dirs, tag=None):
    # each pass (directory) is its own run: its dispatch count can differ from another pass's (the bench sizes
    # its iteration count from a first timing), so every counter is scaled to the dispatch count of the first
    # pass that saw the kernel — the sums stay "per that many dispatches" across passes
    merged = defaultdict(dict)
    ndisp = {}
    for d in dirs:
        tot, disp = load(d)
        for k, v in tot.items():
            n = len(disp[k])
            ndisp.setdefault(k, n)
            scale = ndisp[k] / n if n else 1.0
            merged[k].update({c: x * scale for c, x in v.items()})
    for k, v in sorted(merged.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        out = {"kernel": k[:90], "dispatches": ndisp.get(k, 0)}
        if tag is not None:
            out["pass"] = tag
        out.update({c: int(x) for c, x in sorted(v.items())})
        wc = v.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                      "SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS"):
                if c in v:
                    out[c + "_per_wave_cycle"] = round(v[c] / wc, 4)
        if v.get("SQ_INSTS_LDS"):
            out["lds_bank_conflict_per_lds_inst"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_INSTS_LDS"], 4)
        print(json.dumps(out))


if __name__ == "__main__":
    args = sys.argv[1:]
    tag = None
    if len(args) >= 2 and args[0] == "--tag":  # label every line with its pass (tools/roofline.py ROWS)
        tag, args = args[1], args[2:]
    main(args, tag)
