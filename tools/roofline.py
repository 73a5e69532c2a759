#!/usr/bin/env python3
"""One gfx950 roofline for every search kernel, from counters (profiles/roofline_r5.md is its output).

Peak model (MI355X, stated once; /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters", "LDS"):
  * 256 CUs in 32 shader engines (8 CUs each), 4 SIMD-32 per CU; a wave64 VALU instruction occupies its SIMD
    for 2 cycles, so a CU issues at most 2 wave-instructions per clock. The packed int16 ops the kernels run
    (v_pk_add_u16, v_pk_max_i16, SDWA adds) count as one instruction each.
  * LDS: one array per CU, 256 B per clock for conflict-free ds_read_b64 / ds_read_b128 (128 B per clock for
    ds_read_b32 / _u16 / _u8); SQ_LDS_IDX_ACTIVE counts the array cycles a kernel used, SQ_LDS_BANK_CONFLICT
    the extra cycles of its bank conflicts (both summed over CUs).
  * clock: SQ_BUSY_CYCLES is summed over the 32 shader engines, so BUSY / 32 is the kernel's span in shader
    cycles and BUSY / 32 / t the clock it ran at.
Utilisations are clock-free: VALU = 2 INSTS_VALU / (4 SIMD x 256 CU x span), LDS = LDS_IDX_ACTIVE /
(256 x span). Kernel time and cells come from tools/kernel_bench.py (no counters in that run; the counter run's
own times are longer).

  python tools/roofline.py PMC_SUMMARY.jsonl PMC_RUN_KERNEL_BENCH.log KERNEL_BENCH.log [...] > roofline.md
"""
import json
import sys

CUS, SES = 256, 32

# kernel-bench shape -> the kernel that does its search (the first name match in the counter summary)
SHAPE_KERNEL = {
    "input6": "swipe_direct_kernel<24, 4, false>",
    "input1": "swipe_direct_kernel<24, 16, true>",
    "mid": "short_search_kernel<false, true, true>",
    "input3": "tile16_search_kernel<2, false,",  # prefix: <U, windowed, wide> (the wide entries when they fit)
    "input4": "tile16_search_kernel<8, false,",
    "long20k": "tile16_search_kernel<4, true,",
}


def main(argv):
    pmc = [json.loads(l) for l in open(argv[0]) if l.strip()]

    def shapes(paths):
        out = {}
        for path in paths:
            for line in open(path):
                if line.startswith("{"):
                    d = json.loads(line)
                    out.setdefault(d["shape"], d)
        return out

    pmc_run = shapes(argv[1:2])
    bench = shapes(argv[2:])
    print("| shape | kernel | T cells/s | VALU lane-instr / cell | VALU util | LDS util | LDS conflict share | "
          "clock (GHz, counter run) | waits: s_waitcnt / issue-stall / active (wave cycles) |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---|")
    for shape, kname in SHAPE_KERNEL.items():
        row = next((r for r in pmc if kname in r["kernel"]), None)
        b = bench.get(shape)
        if row is None or b is None:
            continue
        n = row["dispatches"]
        per = {k: v / n for k, v in row.items() if isinstance(v, (int, float)) and k != "dispatches"}
        span = per["SQ_BUSY_CYCLES"] / SES
        valu = 2 * per["SQ_INSTS_VALU"] / (4 * CUS * span)
        lds = per["SQ_LDS_IDX_ACTIVE"] / (CUS * span)
        conflict = per["SQ_LDS_BANK_CONFLICT"] / max(per["SQ_LDS_IDX_ACTIVE"], 1)
        wc = per["SQ_WAVE_CYCLES"]
        waits = f'{per["SQ_WAIT_ANY"] / wc:.2f} / {per["SQ_WAIT_INST_ANY"] / wc:.2f} / {per["SQ_ACTIVE_INST_ANY"] / wc:.2f}'
        # the counter run's kernel time for the clock (its kernel_bench line), the plain run's for throughput
        clock = span / (pmc_run.get(shape, b)["gpu_ms"] * 1e-3) / 1e9
        cells_per_dispatch = b["cells"]
        print(f'| {shape} | `{row["kernel"].split("(")[0]}` | {b["cells_per_s"] / 1e12:.2f} | {per["SQ_INSTS_VALU"] * 64 / cells_per_dispatch:.3f} | '
              f'{valu:.0%} | {lds:.0%} | {conflict:.0%} | {clock:.2f} | {waits} |')


if __name__ == "__main__":
    main(sys.argv[1:])
