#!/usr/bin/env python3
"""Summarise rocprofv3 output of profiles/collect.sh into profiles/.

Writes:
  profiles/<round>/kernel_stats.csv   (copy of the --stats summary)
  profiles/<round>/pmc_per_kernel.csv (avg FETCH_SIZE / WRITE_SIZE per kernel)
  profiles/pmc_summary.json           (read by bench.py for roofline.traffic)

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are KB; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact for
16 B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    """Stable key for our kernels: verify_<len>/compute_<len> are filled in
    by matching the k_fixed template's COMPUTE flag."""
    if "gcs::k_fixed<" in name:
        args = name.split("k_fixed<", 1)[1].split(">", 1)[0].split(",")
        compute = args[2].strip() == "true"
        return ("compute" if compute else "verify") + "_fixed<" + ",".join(a.strip() for a in args) + ">"
    if "gcs::" in name:
        return name.split("(", 1)[0].replace("void ", "")
    return name[:60]


def counters(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = defaultdict(list)
    if not f:
        return out
    for row in csv.DictReader(open(f[0])):
        out[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    return out


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    durations = {}
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        for row in csv.DictReader(open(stats[0])):
            durations[row["Name"]] = float(row["AverageNs"])
    fetch, write = counters(os.path.join(src, "fetch")), counters(os.path.join(src, "write"))
    per = {}
    for (k, c), vals in list(fetch.items()) + list(write.items()):
        e = per.setdefault(k, {})
        e[c] = sum(vals) / len(vals)
        e["dispatches_" + c] = len(vals)
    summary = {"round": rnd, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes)",
               "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = 1/2)",
               "kernels": {}}
    with open(os.path.join(dst, "pmc_per_kernel.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "avg_FETCH_SIZE_KB", "avg_WRITE_SIZE_KB", "hbm_bytes_per_launch",
                    "avg_duration_ns"])
        for k, e in sorted(per.items()):
            if "gcs::" not in k:
                continue
            fs, ws = e.get("FETCH_SIZE"), e.get("WRITE_SIZE")
            hbm = (2 * fs + (ws or 0)) * 1024 if fs is not None else None
            w.writerow([k, fs, ws, hbm, durations.get(k)])
            key = short(k)
            summary["kernels"][key] = {"name": k, "fetch_size_kb": fs, "write_size_kb": ws,
                                       "hbm_bytes_per_launch": hbm,
                                       "avg_duration_ns": durations.get(k)}
            # bench.py looks kernels up as "<verify|compute>_<frame_len>"
            if key.startswith(("verify_fixed<32,3,", "compute_fixed<32,3,")):
                summary["kernels"][key.split("_")[0] + "_1500"] = summary["kernels"][key]
    json.dump(summary, open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w"), indent=1)
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
