#!/usr/bin/env python3
"""Timeline of a short process from rocprofv3 CSV traces (--hip-trace --kernel-trace [--memory-copy-trace]):
every HIP API call longer than a threshold and every kernel / copy, in ms from the first API call.

    python tools/api_timeline.py gpurun_out/hip_wall_trace final [min_ms]
"""
import csv
import os
import sys


def rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def main(d, prefix, min_ms=0.2):
    api = rows(os.path.join(d, f"{prefix}_hip_api_trace.csv"))
    ker = rows(os.path.join(d, f"{prefix}_kernel_trace.csv"))
    cpy = rows(os.path.join(d, f"{prefix}_memory_copy_trace.csv"))
    if not api:
        print(f"no API trace under {d} for {prefix}")
        return 1
    t0 = min(int(r["Start_Timestamp"]) for r in api)
    ev = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if (e - s) / 1e6 >= min_ms:
            ev.append((s, e, f"api tid={r['Thread_Id']} {r['Function']}"))
    for r in ker:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel " + r["Kernel_Name"][:90]))
    for r in cpy:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   f"copy {r.get('Direction', '')} {r.get('Size', '')} B"))
    ev.sort()
    print(f"# {prefix}: {len(api)} API calls, {len(ker)} kernels, {len(cpy)} copies; API calls >= {min_ms} ms shown")
    print(f"# {'start_ms':>9} {'dur_ms':>8}  what")
    for s, e, what in ev:
        print(f"  {(s - t0) / 1e6:9.2f} {(e - s) / 1e6:8.3f}  {what}")
    last = max(e for _, e, _ in ev)
    print(f"# last event ends at {(last - t0) / 1e6:.2f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 0.2))
