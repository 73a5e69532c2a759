"""The measurement tools behind profiles/: their parsers on small synthetic inputs (CPU tier)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_tool(*args):
    return subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=60, cwd=ROOT)


def test_api_timeline(tmp_path):
    # rocprofv3 CSV columns as the tool reads them; times in ns from an arbitrary epoch
    t0 = 1_000_000_000
    with open(tmp_path / "x_hip_api_trace.csv", "w") as f:
        f.write('"Domain","Function","Process_Id","Thread_Id","Correlation_Id","Start_Timestamp","End_Timestamp"\n')
        f.write(f'"HIP","hipGetDeviceCount",1,11,1,{t0},{t0 + 50_000_000}\n')
        f.write(f'"HIP","hipEventCreate",1,11,2,{t0 + 50_000_000},{t0 + 50_010_000}\n')
        f.write(f'"HIP","hipStreamCreateWithFlags",1,12,3,{t0 + 50_100_000},{t0 + 70_100_000}\n')
    with open(tmp_path / "x_kernel_trace.csv", "w") as f:
        f.write('"Kernel_Name","Start_Timestamp","End_Timestamp"\n')
        f.write(f'"swipe_search_kernel<24, 4, 2, false>",{t0 + 71_000_000},{t0 + 71_040_000}\n')
    r = run_tool("tools/api_timeline.py", str(tmp_path), "x")
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if not ln.startswith("#")]
    # calls under 0.2 ms are left out; events in start order, ms from the first call
    assert len(lines) == 3
    assert "hipGetDeviceCount" in lines[0] and lines[0].split()[:2] == ["0.00", "50.000"]
    assert "hipStreamCreateWithFlags" in lines[1] and lines[1].split()[0] == "50.10"
    assert "kernel swipe_search_kernel" in lines[2]
    assert "last event ends at 71.04 ms" in r.stdout
    assert run_tool("tools/api_timeline.py", str(tmp_path), "missing").returncode == 1


def test_step_variance_report(tmp_path):
    # 100 steps, every 10th one 20 % slow; GPU samples over the whole span
    step_ms = [3.0 * (1.2 if i % 10 == 9 else 1.0) for i in range(100)]
    ends, t = [], 0.0
    for ms in step_ms:
        t += ms / 1e3
        ends.append(t)
    with open(tmp_path / "steps.json", "w") as f:
        json.dump({"step_ms": step_ms, "kernel_ms": [m - 0.01 for m in step_ms], "end_time": ends}, f)
    with open(tmp_path / "gpu_samples.jsonl", "w") as f:
        for i in range(40):
            f.write(json.dumps({"t": i * 0.01, "sclk_mhz": 2400, "power_w": 900.0}) + "\n")
    r = run_tool("tools/step_variance_report.py", str(tmp_path))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout[: r.stdout.rindex("}") + 1])
    assert out["steps"] == 100 and out["slow_steps"] == 10
    assert out["bursts"] == {"count": 10, "longest": 1, "mean_len": 1.0}
    assert out["sclk_mhz"]["normal_median"] == 2400


def test_p33_magic_constants():
    # the device decoders' multiply-by-reciprocal constants (swipe_impl.hpp decode_p33_field, lane_length6),
    # exhaustively over their input ranges
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "p33_magic_check.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"
