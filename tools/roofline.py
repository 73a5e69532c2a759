#!/usr/bin/env python3
"""One gfx950 roofline for every search kernel, from counters (profiles/roofline_r6.md is its output; roofline_r5.md the previous round's).

Peak model (MI355X), measured on the box by tools/isa_peak.hip (profiles/roofline_r5/isa_peak.log): 256 CUs of
4 SIMDs; every SIMD holding 8 waves of independent instructions sustains, per CU-clock,
  * 1.69 wave64 VALU instructions of plain 32-bit ops (v_add_u32: 2 cycles per instruction per SIMD);
  * 0.94 of the packed/sub-dword ops the hot loops are made of — v_pk_add_u16, v_pk_max_i16, v_add_u16_sdwa,
    v_add_u32_dpp (row_newbcast), v_readlane_b32: 4 cycles per instruction, HALF the 32-bit rate;
  * 0.48 LDS read instructions (ds_read_b32 / _u16 / _b64, conflict-free: ~2 LDS cycles each; b64 moves 512 B).
  Clock under these loads: 2.25-2.4 GHz (s_memtime over s_memrealtime).
Counters: SQ_INSTS_VALU and SQ_INSTS_LDS are wave-instructions; SQ_BUSY_CYCLES is summed over the 32 shader
engines, so BUSY / 32 is the kernel's span in shader cycles; SQ_LDS_IDX_ACTIVE / SQ_LDS_BANK_CONFLICT are
LDS-array cycles summed over CUs; SQ_WAIT_ANY / SQ_WAVE_CYCLES is the share of wave time spent in s_waitcnt.
The hot loops are almost all packed ops, so "of packed peak" is the VALU bound that applies; a kernel whose
mix holds full-rate ops can exceed 100 % of it. Throughput comes from tools/kernel_bench.py (no counters).

  python tools/roofline.py PMC_SUMMARY.jsonl KERNEL_BENCH.log [...] > roofline.md
"""
import json
import sys

CUS, SES = 256, 32
PEAK_PACKED, PEAK_VALU32, PEAK_LDS = 0.94, 1.69, 0.48  # wave-instructions per CU-clock (isa_peak)

# kernel-bench row (shape, variant) -> the kernel that does its search (a prefix of its name in the summary)
ROWS = [  # shape, kernel_bench variant, kernel name prefix, form, PMC pass (tools/pmc_roofline.sh)
    ("input6", "tile16", "swipe_direct_kernel<20, 4, 0, false>", "device bytes", "p1"),
    ("input6", "wire", "swipe_direct_kernel<20, 4, 2, false>", "device P33 wire", "p4"),
    ("input1", "tile16", "swipe_direct_kernel<20, 12, 0, true>", "device bytes", "p1"),
    ("input1", "wire", "swipe_direct_kernel<20, 12, 2, true>", "device P33 wire", "p4"),
    ("mid", "tile16", "swipe_direct_kernel<64, 24, 0, true>", "device bytes, 24 record words", "p1"),
    ("input3", "tile16", "tile16_search_kernel<4, false, true>", "widened pairs", "p2"),
    ("limits", "tile16", "tile16_slide_kernel<4, 8>", "sliding widened windows", "p2"),
    ("input4", "tile16", "tile16_search_kernel<8, true, true>", "widened windows", "p3"),
    ("long20k", "tile16", "tile16_slide_kernel<4, 8>", "sliding widened windows", "p3"),
    ("heavy3", "tile16", "tile16_search_kernel<2, false, true>", "int16 profile", "p5"),
    ("heavy4", "tile16", "tile16_search_kernel<8, true, true>", "int16 profile, windows", "p5"),
    ("heavylim", "tile16", "tile16_slide_kernel<4, 8>", "int16 profile, sliding widened windows", "p6"),
]


def main(argv):
    pmc = [json.loads(l) for l in open(argv[0]) if l.strip()]
    bench = {}
    for path in argv[1:]:
        for line in open(path):
            if line.startswith("{"):
                d = json.loads(line)
                variant = "wire" if d["variant"].startswith("wire-p33") else d["variant"]
                bench.setdefault((d["shape"], variant), d)
    print("| shape | path | kernel | T cells/s | VALU lane-instr / cell | VALU wave-instr / CU-clock | of packed peak | "
          "LDS wave-instr / CU-clock | of LDS peak | LDS conflict share | s_waitcnt share |")
    print("|---|---|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for shape, variant, kname, path, tag in ROWS:
        rows = [r for r in pmc if kname in r["kernel"] and r.get("pass", tag) == tag]
        b = bench.get((shape, variant))
        if not rows or b is None:
            continue
        row = rows[0]
        n = row["dispatches"]
        per = {k: v / n for k, v in row.items() if isinstance(v, (int, float)) and k != "dispatches"}
        span = per["SQ_BUSY_CYCLES"] / SES
        valu = per["SQ_INSTS_VALU"] / (CUS * span)
        lds = per["SQ_INSTS_LDS"] / (CUS * span)
        conflict = per.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(per.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0)
        waits = per["SQ_WAIT_ANY"] / per["SQ_WAVE_CYCLES"]
        print(f'| {shape} | {path} | `{row["kernel"].split("(")[0].replace("void moc::dev::", "")}` | '
              f'{b["cells_per_s"] / 1e12:.2f} | {per["SQ_INSTS_VALU"] * 64 / b["cells"]:.2f} | {valu:.2f} | '
              f'{valu / PEAK_PACKED:.0%} | {lds:.2f} | {lds / PEAK_LDS:.0%} | {conflict:.0%} | {waits:.0%} |')


if __name__ == "__main__":
    main(sys.argv[1:])
