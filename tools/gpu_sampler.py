#!/usr/bin/env python3
"""Samples one GPU's clocks, power and temperature from the amdgpu driver's sysfs files (no SMI library,
no root) every --period seconds until killed or --duration ends, as JSON lines with wall-clock times, so a
benchmark's per-step times (bench.py --dump-steps: "end_time") can be lined up with what the GPU did.

    python tools/gpu_sampler.py --bus 0000:5d:00.0 --period 0.02 --out gpurun_out/samples.jsonl &

The card is found by its PCIe address (bench.py reports rank_pci_bus); without --bus the first card with a
hwmon directory is used. Fields: t (time.time()), sclk_mhz / mclk_mhz (the active DPM level of
pp_dpm_sclk / pp_dpm_mclk), power_w (power1_average or power1_input), temp_c (temp1_input), busy_pct
(gpu_busy_percent) — each only when the driver exposes it.
"""
import argparse
import glob
import json
import os
import re
import sys
import time


def find_card(bus):
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        real = os.path.realpath(dev)
        if bus and os.path.basename(real).lower() != bus.lower():
            continue
        if glob.glob(os.path.join(dev, "hwmon", "hwmon*")) or os.path.exists(os.path.join(dev, "pp_dpm_sclk")):
            return dev
    return None


def active_level(path):
    try:
        with open(path) as f:
            for line in f:
                if line.rstrip().endswith("*"):
                    m = re.search(r"(\d+)\s*[mM]hz", line)
                    return int(m.group(1)) if m else None
    except OSError:
        return None
    return None


def read_num(path, scale=1.0):
    try:
        with open(path) as f:
            return float(f.read().strip()) * scale
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bus", default="")
    ap.add_argument("--period", type=float, default=0.02)
    ap.add_argument("--duration", type=float, default=600.0)
    ap.add_argument("--out", default="-")
    args = ap.parse_args()
    dev = find_card(args.bus)
    out = sys.stdout if args.out == "-" else open(args.out, "w", buffering=1)
    if dev is None:
        print(json.dumps({"error": f"no amdgpu card for bus {args.bus!r}"}), file=out, flush=True)
        return 1
    hw = (glob.glob(os.path.join(dev, "hwmon", "hwmon*")) or [None])[0]
    print(json.dumps({"card": os.path.realpath(dev), "hwmon": hw}), file=out, flush=True)
    end = time.time() + args.duration
    while time.time() < end:
        s = {"t": round(time.time(), 4), "sclk_mhz": active_level(os.path.join(dev, "pp_dpm_sclk")),
             "mclk_mhz": active_level(os.path.join(dev, "pp_dpm_mclk")),
             "busy_pct": read_num(os.path.join(dev, "gpu_busy_percent"))}
        if hw:
            p = read_num(os.path.join(hw, "power1_average"), 1e-6)
            s["power_w"] = p if p is not None else read_num(os.path.join(hw, "power1_input"), 1e-6)
            s["temp_c"] = read_num(os.path.join(hw, "temp1_input"), 1e-3)
            f = read_num(os.path.join(hw, "freq1_input"), 1e-6)
            if f is not None:
                s["sclk_hwmon_mhz"] = f
        print(json.dumps(s), file=out, flush=True)
        time.sleep(args.period)
    return 0


if __name__ == "__main__":
    sys.exit(main())
