#!/usr/bin/env python3
"""Turn a scripts/gpu_profile.sh output directory into profiles/pmc_traffic.json:
per-kernel HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (separate --pmc
passes), corrected with the calibration stream of tools/calib_fetch.hip
(MI355X_MICROARCH.md §HBM: FETCH_SIZE reports 1/2 of a coalesced stream)."""
import collections
import csv
import json
import sys


def agg(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def readable(rocprof_name):
    """'void gcmx::k_step_tx2<2, 512, true, true, false>(...)' -> the library's
    symbol form 'k_step_tx2<2, 512, KF0, UNI, !FACES>' (gcmx_profile_kernel)."""
    import re
    m = re.search(r"(k_step_tx2|k_fused_xyz)<([^>]*)>", rocprof_name)
    if not m:
        return rocprof_name
    a = [x.strip() for x in m.group(2).split(",")]
    flags = ["KF0", "UNI", "FACES"]
    out = a[:2] + [(f if v == "true" else "!" + f) for f, v in zip(flags, a[2:5])]
    # k_step_tx2's HET and ZS flags appear in the library's name only when set
    out += [f for f, v in zip(["HET", "ZS"], a[5:7]) if v == "true"]
    if "xyz_fma::" in rocprof_name:  # the contracted build (gcmx_set_fp_mode), as the library names it
        out.append("FMA")
    return f"{m.group(1)}<{', '.join(out)}>"


def main(prof_dir, out, n=512, lib_path="gcm_amd/lib/libgcmx.so", calib_json=None):
    f = agg(f"{prof_dir}/fetch/run_counter_collection.csv", "FETCH_SIZE")
    w = agg(f"{prof_dir}/write/run_counter_collection.csv", "WRITE_SIZE")
    true = 8 * (1 << 30)
    try:
        cf = agg(f"{prof_dir}/calib_fetch/run_counter_collection.csv", "FETCH_SIZE")
        cw = agg(f"{prof_dir}/calib_write/run_counter_collection.csv", "WRITE_SIZE")
        r8 = [v for k, v in cf.items() if k.startswith("read8")][0] * 1024
        w8 = [v for k, v in cw.items() if k.startswith("write8")][0] * 1024
    except (FileNotFoundError, IndexError):  # reuse the stored calibration run
        old = json.load(open(calib_json or out))["calibration"]
        r8, w8 = old["read8_fetch_bytes"], old["write8_write_bytes"]
    ff, wf = true / r8, true / w8
    alg = 144 * n ** 3
    import hashlib
    sha = hashlib.sha256(open(lib_path, "rb").read()).hexdigest()
    z = min(t for t in (64, 128, 256, 512, 1024) if t >= n)  # the launch's ZT
    res = {"n": n, "ranks": 1, "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, {prof_dir}",
           "lib_sha256": sha,
           "calibration": {"tool": "tools/calib_fetch.hip", "true_bytes": true,
                           "read8_fetch_bytes": r8, "fetch_factor": ff,
                           "write8_write_bytes": w8, "write_factor": wf},
           "kernels": {}}
    # bench.py's bucket "fused_xyz" is the one-pass step: k_step_tx2 (default) or
    # k_fused_xyz; rows longer than 512 run the z split, k_step_tx2<2, 512, ..., ZS>
    # followed by k_zseam in the same bucket, so their bytes add up
    zsplit = ("fused_xyz", "k_step_tx2<2, 512, true, true, false, false, true>", "k_zseam<2")
    for short, frag, *extra in (("march_x", "k_march<0, 2"), ("fused_yz", f"k_fused_yz<2, {z}"),
                                ("fused_xyz", f"k_fused_xyz<2, {z}"), ("fused_xyz", f"k_step_tx2<2, {z}"),
                                *((zsplit,) if n > 512 else ())):
        fks = [v for k, v in f.items() if frag in k]
        wks = [v for k, v in w.items() if frag in k]
        if not fks or not wks:
            continue
        fk = fks[0] * 1024 * ff
        wk = wks[0] * 1024 * wf
        for e in extra:  # the seam kernel's bytes, same launches
            fk += sum(v for k, v in f.items() if e in k) * 1024 * ff
            wk += sum(v for k, v in w.items() if e in k) * 1024 * wf
        full = [k for k in f if frag in k][0]
        res["kernels"][short] = {"symbol": readable(full), "rocprof_name": full,
                                 "fetch_bytes_per_launch": fk, "write_bytes_per_launch": wk,
                                 "hbm_bytes_per_launch": fk + wk,
                                 "algorithmic_bytes_per_launch": alg,
                                 "traffic_over_algorithmic": (fk + wk) / alg}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    # pmc_traffic.py PROF_DIR OUT.json [N] [CALIBRATION.json: reuse its stored calibration]
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 512,
         calib_json=sys.argv[4] if len(sys.argv) > 4 else None)
