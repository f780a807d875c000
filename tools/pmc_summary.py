"""Fold rocprofv3 CSV output (kernel stats + FETCH_SIZE / WRITE_SIZE passes)
into one JSON summary for the rollout kernel.

Units/corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so fetch bytes = 2 x 1024 x FETCH_SIZE;
write bytes = 1024 x WRITE_SIZE.  Both are per dispatch.
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_rollout"


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def counter(d, name):
    vals = []
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        kn = r.get("Kernel_Name", "")
        if KERNEL in kn and r.get("Counter_Name") == name:
            vals.append(float(r["Counter_Value"]))
    return vals


def main(d):
    stats = {}
    for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                            "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
    roll = {k: v for k, v in stats.items() if KERNEL in k}
    fetch = counter(os.path.join(d, "pmc_fetch"), "FETCH_SIZE")
    write = counter(os.path.join(d, "pmc_write"), "WRITE_SIZE")
    out = {"kernel_stats": stats, "rollout": roll}
    if fetch and write:
        f = sum(fetch) / len(fetch)
        w = sum(write) / len(write)
        out["fetch_size_kib_per_launch"] = f
        out["write_size_kib_per_launch"] = w
        out["hbm_bytes_per_launch"] = 2 * 1024 * f + 1024 * w
        out["hbm_bytes_note"] = "2*1024*FETCH_SIZE + 1024*WRITE_SIZE (gfx950 FETCH_SIZE half-count correction)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
