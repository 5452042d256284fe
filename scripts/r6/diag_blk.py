#!/usr/bin/env python3
"""Per-block timing of one k_step_tx2 launch (tuning build with GCMX_TX2_BLKT=1,
GCMX_LIB=gcm_amd/lib/tune/blkt/libgcmx.so): how long each block runs, when it
starts and ends, how evenly the CUs finish -- the headroom a dynamic (work-
stealing) assignment of row chunks could recover.

    GCMX_LIB=gcm_amd/lib/tune/blkt/libgcmx.so python scripts/r6/diag_blk.py [N] [--rows R] [--out file.npz]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import gcm_amd  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="?", default=512)
ap.add_argument("--rows", type=int, default=0)
ap.add_argument("--launches", type=int, default=3)
ap.add_argument("--out", default="")
a = ap.parse_args()
N = a.n
L = gcm_amd.gcmx.lib()
f = L.gcmx_diag_blk_fma
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
U, U1, Lm = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
c = gcm_amd.Context(3, 2, [N, N, N], device=0)
c.set_materials(U[None], U1[None], Lm[None])
if a.rows:
    c.set_schedule(gcm_amd.SCHED_AUTO, a.rows)
c.fill_random([N, N, N], 0x5EED)
for _ in range(3):
    c.step(0.9)
c.sync()
t = np.zeros((8192, 8, 2), np.uint64)
hw = np.zeros(8192, np.uint32)
assert f(t.ctypes.data, hw.ctypes.data) == 0
saved = []
for k in range(a.launches):
    c.step(0.9)
    c.sync()
    assert f(t.ctypes.data, hw.ctypes.data) == 0
    nb = int((t[:, 0, 1] > 0).sum())
    tt = t[:nb].astype(np.int64)
    w = tt[:, :, 1] > 0  # waves present
    st = np.where(w, tt[:, :, 0], np.iinfo(np.int64).max).min(1)
    en = np.where(w, tt[:, :, 1], 0).max(1)
    t0 = st.min()
    st, en = (st - t0) / 100.0, (en - t0) / 100.0  # microseconds (100 MHz)
    dur = en - st
    span = en.max()
    cu = (hw[:nb] >> 8) & 0xF
    sh = (hw[:nb] >> 12) & 0x1
    se = (hw[:nb] >> 13) & 0x7
    xcd = np.arange(nb) % 8
    slot = ((xcd * 8 + se) * 2 + sh) * 16 + cu
    busy = {}
    for s_, d_ in zip(slot, dur):
        busy[int(s_)] = busy.get(int(s_), 0.0) + d_
    bv = np.array(list(busy.values()))
    xcd_end = [float(en[xcd == i].max()) for i in range(8)]
    wave_skew = (np.where(w, tt[:, :, 1], 0).max(1) - np.where(w, tt[:, :, 1], np.iinfo(np.int64).max).min(1)) / 100.0
    rec = {"n": N, "launch": k, "blocks": nb, "distinct_slots": len(busy), "span_us": round(float(span), 1),
           "dur_us": {"min": round(float(dur.min()), 1), "p10": round(float(np.percentile(dur, 10)), 1),
                      "median": round(float(np.median(dur)), 1), "p90": round(float(np.percentile(dur, 90)), 1),
                      "max": round(float(dur.max()), 1)},
           "start_us": {"median": round(float(np.median(st)), 1), "max": round(float(st.max()), 1)},
           "end_us": {"p10": round(float(np.percentile(en, 10)), 1), "median": round(float(np.median(en)), 1),
                      "max": round(float(en.max()), 1)},
           "slot_busy_us": {"mean": round(float(bv.mean()), 1), "min": round(float(bv.min()), 1),
                            "max": round(float(bv.max()), 1)},
           "xcd_end_us": [round(v, 1) for v in xcd_end],
           "wave_end_skew_us": {"median": round(float(np.median(wave_skew)), 1), "max": round(float(wave_skew.max()), 1)},
           "mean_busy_over_span": round(float(bv.mean() / span), 4)}
    print(json.dumps(rec), flush=True)
    saved.append((tt, hw[:nb].copy()))
if a.out:
    np.savez_compressed(a.out, **{f"t{k}": s[0] for k, s in enumerate(saved)}, **{f"hw{k}": s[1] for k, s in enumerate(saved)})
c.close()
