#!/usr/bin/env python3
"""Runs a command (a probe binary) while sampling the GPU's power and sclk
from amdgpu sysfs (tools/box_state.py) every 20 ms, then attributes the samples
to the probe's variants by the CLOCK_MONOTONIC spans they print ("[mono t0 t1]").
Measurement only.  Usage: power_probe.py OUTFILE -- CMD ARGS..."""
import json
import os
import re
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import box_state  # noqa: E402


def main():
    out = sys.argv[1]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    dev = box_state.card_dir(0)
    hw = box_state._hwmon(dev) if dev else None
    samples, stop = [], threading.Event()

    def run():
        while not stop.is_set():
            t = time.monotonic()
            p = box_state._power(hw)
            d = box_state._dpm(box_state._read(os.path.join(dev, "pp_dpm_sclk"))) if dev else None
            samples.append((t, p, d["current"] if d else None))
            stop.wait(0.02)

    th = threading.Thread(target=run, daemon=True)
    if dev:
        th.start()
    r = subprocess.run(cmd, capture_output=True, text=True)
    stop.set()
    if dev:
        th.join(2)
    rows = []
    for line in r.stdout.splitlines():
        m = re.search(r"\[mono ([0-9.]+) ([0-9.]+)\]", line)
        rec = {"line": re.sub(r"\s*\[mono.*\]", "", line)}
        if m:
            t0, t1 = float(m.group(1)), float(m.group(2))
            # skip the first 30 % of the span (the power average lags)
            ts = t0 + 0.3 * (t1 - t0)
            ss = [(p, c) for (t, p, c) in samples if ts <= t <= t1 and p is not None]
            if ss:
                pw = sorted(p for p, _ in ss)
                cl = sorted(int(c[:-3]) for _, c in ss if c and c.endswith("Mhz"))
                rec.update({"span_s": round(t1 - t0, 3), "samples": len(ss), "power_w_median": pw[len(pw) // 2],
                            "sclk_mhz_median": cl[len(cl) // 2] if cl else None})
        rows.append(rec)
        print(rec["line"] + (f"  | {rec.get('power_w_median')} W, sclk {rec.get('sclk_mhz_median')} MHz, "
                             f"{rec.get('samples')} samples" if "samples" in rec else ""))
    with open(out, "w") as f:
        json.dump({"cmd": cmd, "rc": r.returncode, "rows": rows, "stderr": r.stderr[-2000:]}, f, indent=1)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
