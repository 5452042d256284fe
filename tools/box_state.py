"""What the box a bench line ran on looks like, from the amdgpu sysfs of the GPU
the process uses (find what separates the 4.20 ms boxes from
the 3.97 ms ones).  Measurement only; read-only sysfs access, nothing here
touches the GPU.

* `static_state(device)`: partition modes, firmware / VBIOS versions, power cap,
  DPM level tables (with the '*' level at the time of the read), the board's
  unique id (to recognise a box seen before), temperatures.
* `Sampler(device)`: a thread that samples the current DPM levels (sclk, mclk,
  fclk, socclk), power and temperatures every `period` seconds while the timed
  repetitions run (the main thread waits inside ctypes calls, which release
  the GIL), summarised per quantity.
"""
import glob
import os
import re
import threading
import time


def _read(path, limit=4096):
    try:
        with open(path, "r", errors="replace") as f:
            return f.read(limit).strip()
    except Exception:
        return None


def card_dir(device=0):
    """The /sys/class/drm/cardN/device directory of HIP device `device`, matched by
    PCI address (torch's device properties); None when it cannot be found."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device)
        want = "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    except Exception:
        want = None
    cards = sorted(glob.glob("/sys/class/drm/card[0-9]*/device"))
    amd = []
    for c in cards:
        ue = _read(os.path.join(c, "uevent")) or ""
        if "DRIVER=amdgpu" not in ue:
            continue
        slot = re.search(r"PCI_SLOT_NAME=(\S+)", ue)
        slot = slot.group(1).lower() if slot else ""
        amd.append((c, slot))
        if want and slot.startswith(want):
            return c
    return amd[0][0] if len(amd) == 1 else None


def _dpm(text):
    """pp_dpm_* table -> {'levels': [...], 'current': '...'}"""
    if not text:
        return None
    levels, cur = [], None
    for line in text.splitlines():
        m = re.match(r"\s*(\d+):\s*(\S+)\s*(\*)?", line)
        if m:
            levels.append(m.group(2))
            if m.group(3):
                cur = m.group(2)
    return {"levels": levels, "current": cur}


def _hwmon(dev):
    hw = sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*")))
    return hw[0] if hw else None


def _num(path, scale=1.0):
    v = _read(path)
    try:
        return float(v) * scale
    except (TypeError, ValueError):
        return None


def _temps(hw):
    out = {}
    if not hw:
        return out
    for f in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
        lab = _read(f.replace("_input", "_label")) or os.path.basename(f)
        out[lab] = _num(f, 1e-3)
    return out


def _power(hw):
    if not hw:
        return None
    for name in ("power1_average", "power1_input"):
        v = _num(os.path.join(hw, name), 1e-6)
        if v is not None:
            return v
    return None


def static_state(device=0):
    dev = card_dir(device)
    if dev is None:
        return {"sysfs": "no amdgpu card directory found for this device"}
    hw = _hwmon(dev)
    fw = {}
    for f in sorted(glob.glob(os.path.join(dev, "fw_version", "*"))):
        v = _read(f)
        if v is not None:
            fw[os.path.basename(f)] = v
    st = {
        "card": dev,
        "unique_id": _read(os.path.join(dev, "unique_id")),
        "serial_number": _read(os.path.join(dev, "serial_number")),
        "vbios_version": _read(os.path.join(dev, "vbios_version")),
        "current_memory_partition": _read(os.path.join(dev, "current_memory_partition")),
        "available_memory_partition": _read(os.path.join(dev, "available_memory_partition")),
        "current_compute_partition": _read(os.path.join(dev, "current_compute_partition")),
        "available_compute_partition": _read(os.path.join(dev, "available_compute_partition")),
        "power_dpm_force_performance_level": _read(os.path.join(dev, "power_dpm_force_performance_level")),
        "pp_power_profile_mode": (_read(os.path.join(dev, "pp_power_profile_mode")) or "")[:600] or None,
        "power_cap_w": _num(os.path.join(hw, "power1_cap"), 1e-6) if hw else None,
        "power_cap_max_w": _num(os.path.join(hw, "power1_cap_max"), 1e-6) if hw else None,
        "power_cap_default_w": _num(os.path.join(hw, "power1_cap_default"), 1e-6) if hw else None,
        "idle_power_w": _power(hw),
        "idle_temps_c": _temps(hw),
        "mem_info_vram_total": _read(os.path.join(dev, "mem_info_vram_total")),
        "fw_version": fw,
    }
    for clk in ("sclk", "mclk", "fclk", "socclk", "vclk", "dclk"):
        st["pp_dpm_" + clk] = _dpm(_read(os.path.join(dev, "pp_dpm_" + clk)))
    gm = os.path.join(dev, "gpu_metrics")
    try:
        with open(gm, "rb") as f:
            raw = f.read(4)
        if len(raw) >= 4:  # metrics_table_header: u16 structure_size, u8 format, u8 content
            st["gpu_metrics_header"] = {"size": raw[0] | raw[1] << 8, "format_revision": raw[2],
                                        "content_revision": raw[3]}
    except Exception:
        pass
    return st


class Sampler:
    """Samples the current DPM levels, power and temperatures in a thread."""

    CLKS = ("sclk", "mclk", "fclk", "socclk")

    def __init__(self, device=0, period=0.05):
        self.dev = card_dir(device)
        self.hw = _hwmon(self.dev) if self.dev else None
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self._t = None

    def _one(self):
        s = {"t": time.perf_counter()}
        for clk in self.CLKS:
            d = _dpm(_read(os.path.join(self.dev, "pp_dpm_" + clk)))
            s[clk] = d["current"] if d else None
        s["power_w"] = _power(self.hw)
        s["temps"] = _temps(self.hw)
        return s

    def _run(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._one())
            except Exception:
                pass
            self._stop.wait(self.period)

    def start(self):
        if self.dev is None:
            return self
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()
        return self

    def stop(self):
        if self._t is None:
            return {"samples": 0, "note": "no amdgpu card directory found"}
        self._stop.set()
        self._t.join(timeout=2.0)
        ss = self.samples
        out = {"samples": len(ss), "period_s": self.period}
        for clk in self.CLKS:
            vals = [s[clk] for s in ss if s.get(clk)]
            hist = {}
            for v in vals:
                hist[v] = hist.get(v, 0) + 1
            out[clk] = hist
        pw = sorted(s["power_w"] for s in ss if s.get("power_w") is not None)
        if pw:
            out["power_w"] = {"median": round(pw[len(pw) // 2], 1), "max": round(pw[-1], 1)}
        temps = {}
        for s in ss:
            for k, v in (s.get("temps") or {}).items():
                if v is not None:
                    temps.setdefault(k, []).append(v)
        out["temps_c_max"] = {k: round(max(v), 1) for k, v in temps.items()}
        return out
