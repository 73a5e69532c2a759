#!/usr/bin/env python3
"""Attributes the headline bench's slow steps (tools/step_variance.sh): per-step host and kernel times from
bench.py --dump-steps, lined up with the GPU's sampled clocks, power and temperature (tools/gpu_sampler.py).

A step is slow when its host time exceeds 1.05 x the median. For slow and normal steps the report compares
the kernel's own time (events: is the GPU slower, or the host between kernels?) and the GPU samples inside
the step's time window (clocks, power, temperature), and lists the bursts of consecutive slow steps.

    python tools/step_variance_report.py gpurun_out/step_variance
"""
import json
import os
import sys

import numpy as np


def load(d):
    with open(os.path.join(d, "steps.json")) as f:
        steps = json.load(f)
    samples = []
    path = os.path.join(d, "gpu_samples.jsonl")
    if os.path.exists(path):
        with open(path) as f:
            for line in f:
                try:
                    s = json.loads(line)
                except ValueError:
                    continue
                if "t" in s:
                    samples.append(s)
    return steps, samples


def main(d):
    steps, samples = load(d)
    sms = np.array(steps["step_ms"])
    kms = np.array(steps["kernel_ms"])
    ends = np.array(steps.get("end_time", []))
    p50 = float(np.median(sms))
    slow = sms > 1.05 * p50
    out = {"steps": int(sms.size), "step_ms_p50": round(p50, 4), "step_ms_p99": round(float(np.percentile(sms, 99)), 4),
           "p99_over_p50": round(float(np.percentile(sms, 99)) / p50, 4), "slow_steps": int(slow.sum()),
           "kernel_ms_p50": round(float(np.median(kms)), 4), "kernel_ms_p99": round(float(np.percentile(kms, 99)), 4),
           "kernel_ms_slow_steps_median": round(float(np.median(kms[slow])), 4) if slow.any() else None,
           "host_gap_ms_p50": round(float(np.median(sms - kms)), 4),
           "host_gap_ms_slow_steps_median": round(float(np.median((sms - kms)[slow])), 4) if slow.any() else None}
    # bursts of consecutive slow steps
    bursts, run = [], 0
    for s in slow:
        if s:
            run += 1
        elif run:
            bursts.append(run)
            run = 0
    if run:
        bursts.append(run)
    out["bursts"] = {"count": len(bursts), "longest": max(bursts) if bursts else 0,
                     "mean_len": round(float(np.mean(bursts)), 2) if bursts else 0}
    # GPU samples in slow vs normal step windows
    if samples and ends.size == sms.size:
        starts = ends - sms / 1e3
        ts = np.array([s["t"] for s in samples])
        lo = np.searchsorted(ts, starts - 0.005)
        hi = np.searchsorted(ts, ends + 0.005, side="right")
        for key in ("sclk_mhz", "mclk_mhz", "power_w", "temp_c", "sclk_hwmon_mhz"):
            vs, vn = [], []
            for i in range(sms.size):
                vals = [samples[j][key] for j in range(lo[i], hi[i]) if samples[j].get(key) is not None]
                (vs if slow[i] else vn).extend(vals)
            if vs or vn:
                out[key] = {"slow_median": float(np.median(vs)) if vs else None,
                            "normal_median": float(np.median(vn)) if vn else None,
                            "slow_min": float(np.min(vs)) if vs else None, "normal_min": float(np.min(vn)) if vn else None,
                            "samples_slow": len(vs), "samples_normal": len(vn)}
        out["gpu_samples"] = len(samples)
        span = samples[-1]["t"] - samples[0]["t"] if len(samples) > 1 else 0
        out["sample_period_ms"] = round(1e3 * span / max(len(samples) - 1, 1), 2)
    print(json.dumps(out, indent=1))
    for f in ("host_before.txt", "host_after.txt"):
        p = os.path.join(d, f)
        if os.path.exists(p):
            print(f"--- {f}")
            with open(p) as fh:
                print(fh.read().rstrip())
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/step_variance"))
