#!/usr/bin/env python3
"""What torch.cuda sees in a process that also loads libgcmx (bench.py's rank
picks its device with torch.cuda.device_count() after importing gcm_amd)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
stage = sys.argv[1]
import torch  # noqa: E402
if stage == "fresh":
    print("fresh: device_count", torch.cuda.device_count(), "is_available", torch.cuda.is_available(), flush=True)
elif stage == "after_import":
    import gcm_amd  # noqa: F401
    gcm_amd.gcmx.lib()
    print("after lib load: device_count", torch.cuda.device_count(), flush=True)
    print("after lib load: is_available", torch.cuda.is_available(), flush=True)
elif stage == "after_ctx":
    import gcm_amd
    c = gcm_amd.Context(3, 2, [4, 8, 64], device=0)
    print("after ctx: device_count", torch.cuda.device_count(), flush=True)
    print("after ctx: is_available", torch.cuda.is_available(), flush=True)
    c.close()
elif stage == "torch_first":
    print("torch first: is_available", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
    x = torch.ones(4, device="cuda:0")
    import gcm_amd
    c = gcm_amd.Context(3, 2, [4, 8, 64], device=0)
    print("torch first, then ctx ok; sum", float(x.sum()), flush=True)
    c.close()
for lib in ("libamdhip64", "libhsa-runtime64", "librccl"):
    maps = [ln.split()[-1] for ln in open("/proc/self/maps") if lib in ln]
    print(" ", lib, sorted(set(maps)))
