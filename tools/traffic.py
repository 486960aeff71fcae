#!/usr/bin/env python3
"""HBM traffic of fw::k_ingest from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

Usage: traffic.py <workload> <fetch_dir> <write_dir> <out_json>

<fetch_dir> / <write_dir> hold the counter-collection CSVs of two separate runs of
    rocprofv3 --pmc FETCH_SIZE  -- python3 bench.py --workload W --calibrate-traffic ...
    rocprofv3 --pmc WRITE_SIZE  -- python3 bench.py --workload W --calibrate-traffic ...
(FETCH_SIZE uses 3 of the 4 TCC slots and WRITE_SIZE 2, so they cannot share a pass).

Corrections: FETCH_SIZE/WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE under-reports wide
streaming reads (the guide measures exactly 1/2 at 16 B/lane; other widths are uncalibrated),
so the read scale is calibrated on this run's own known-byte launch: fw::k_key_groups over
2^28 int64 keys (bench.py --calibrate-traffic) reads exactly 2 GiB with the same 8-B/lane
global loads k_ingest uses and writes 1 GiB.  WRITE_SIZE is taken at face value for k_ingest's
16-B/lane staged stores (exact per the guide); the 4-B/lane calibration write is reported only.
Only the timed launches of the operator are averaged (all k_ingest dispatches of the run: the
warmup handle runs the same kernel on the same stream, so every dispatch is a full batch).
"""
import csv
import glob
import json
import os
import sys

CAL_READ = (1 << 28) * 8
CAL_WRITE = (1 << 28) * 4


def per_kernel(d, counter):
    vals = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            # the flush + fire kernel: k_merge_fire, or k_merge_hopb for SQL HOP with block state
            key = "k_ingest" if "k_ingest" in name else "k_key_groups" if "k_key_groups" in name else \
                  "k_merge_fire" if ("k_merge_fire" in name or "k_merge_hopb" in name) else None
            if key:
                vals.setdefault(key, []).append(float(row["Counter_Value"]))
    return vals


def main():
    wl, fdir, wdir, out = sys.argv[1:5]
    fv, wv = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    cal_f = fv["k_key_groups"][0] * 1024.0
    cal_w = wv["k_key_groups"][0] * 1024.0
    read_scale = CAL_READ / cal_f
    ing_f = sum(fv["k_ingest"]) / len(fv["k_ingest"]) * 1024.0
    ing_w = sum(wv["k_ingest"]) / len(wv["k_ingest"]) * 1024.0
    res = {
        "workload": wl,
        "n_gpus": 1,            # tools/measure.sh runs the PMC passes at N = 1 with the default plan
        "plan": "one-phase",
        "k_ingest_hbm_bytes_per_launch": ing_f * read_scale + ing_w,
        "k_ingest_read_bytes_per_launch": ing_f * read_scale,
        "k_ingest_write_bytes_per_launch": ing_w,
        "k_ingest_launches": len(fv["k_ingest"]),
        "raw_fetch_size_bytes_per_launch": ing_f,
        "calibration": {"kernel": "fw::k_key_groups, 2^28 int64 keys",
                        "known_read_bytes": CAL_READ, "fetch_size_bytes": cal_f, "read_scale": read_scale,
                        "known_write_bytes": CAL_WRITE, "write_size_bytes": cal_w},
    }
    if "k_merge_fire" in fv and "k_merge_fire" in wv:
        res["k_merge_fire_hbm_bytes_per_launch"] = (sum(fv["k_merge_fire"]) / len(fv["k_merge_fire"]) * 1024.0 * read_scale
                                                   + sum(wv["k_merge_fire"]) / len(wv["k_merge_fire"]) * 1024.0)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
