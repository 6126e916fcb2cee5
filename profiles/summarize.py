#!/usr/bin/env python3
"""Summarise the rocprofv3 output of profiles/collect.sh into profiles/.

    python profiles/summarize.py gpurun_out/prof_<round> <round>

Inputs (under the source directory, one rocprofv3 run each):
  bench/   --kernel-trace --stats of `bench.py` (the bench line's own command)
  trace/   --kernel-trace of profiles/pmc_configs.py
  fetch/   --pmc FETCH_SIZE of the same command
  write/   --pmc WRITE_SIZE of the same command
  manifest.json   pmc_configs.py's label of every gcs launch, in order

Writes:
  profiles/<round>/kernel_stats.csv    the bench run's --stats summary
  profiles/<round>/kernel_stats_extras.csv  the same for bench.py with its side
                                       measurements (their kernels' averages)
  profiles/<round>/pmc_configs.csv     per configuration: kernel, launches,
                                       FETCH/WRITE KB, HBM bytes, duration
  profiles/pmc_summary.json            read by bench.py (roofline.traffic)

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: both counters
are KB; on gfx950 FETCH_SIZE counts half the bytes of a wide coalesced
streaming read (MI355X_MICROARCH.md, HBM / rocprofv3 section); WRITE_SIZE is
exact for 16 B-per-lane streaming stores.

Pairing: every launcher of libmtcp_gpucsum launches one kernel, and
pmc_configs.py launches on one stream, so the k-th gcs:: launch (by
Dispatch_Id) is the k-th manifest label.  A count mismatch is an
error.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(pattern):
    f = glob.glob(pattern, recursive=True)
    return f[0] if f else None


def gcs_rows(path, key):
    """gcs:: rows of a rocprofv3 CSV sorted by dispatch, grouped per dispatch."""
    rows = [r for r in csv.DictReader(open(path)) if "gcs::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r[key]))
    return rows


def per_dispatch_counter(d, counter):
    f = one(os.path.join(d, "**", "*counter_collection.csv"))
    if not f:
        return None
    out = {}
    for r in gcs_rows(f, "Dispatch_Id"):
        if r["Counter_Name"] == counter:
            did = int(r["Dispatch_Id"])
            out[did] = out.get(did, 0.0) + float(r["Counter_Value"])   # sum over dimensions
            out.setdefault(("name", did), r["Kernel_Name"])
    ids = sorted(k for k in out if not isinstance(k, tuple))
    return [(out[("name", i)], out[i]) for i in ids]


def per_dispatch_duration(d):
    f = one(os.path.join(d, "**", "*kernel_trace.csv"))
    if not f:
        return None
    return [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in gcs_rows(f, "Dispatch_Id")]


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    stats = one(os.path.join(src, "bench", "**", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    stats = one(os.path.join(src, "bench_extras", "**", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats, os.path.join(dst, "kernel_stats_extras.csv"))
    labels = json.load(open(os.path.join(src, "manifest.json")))["labels"]
    series = {"FETCH_SIZE": per_dispatch_counter(os.path.join(src, "fetch"), "FETCH_SIZE"),
              "WRITE_SIZE": per_dispatch_counter(os.path.join(src, "write"), "WRITE_SIZE"),
              "duration_ns": per_dispatch_duration(os.path.join(src, "trace"))}
    acc = defaultdict(lambda: defaultdict(list))
    names = {}
    for what, s in series.items():
        if s is None:
            continue
        if len(s) != len(labels):
            raise SystemExit(f"{what}: {len(s)} gcs dispatches vs {len(labels)} manifest labels")
        for lab, (name, val) in zip(labels, s):
            if lab == "setup":
                continue
            if names.setdefault(lab, name) != name:
                raise SystemExit(f"{lab}: kernel {name} vs {names[lab]}")
            acc[lab][what].append(val)
    summary = {
        "round": rnd,
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE and --kernel-trace, separate runs of "
                  "profiles/pmc_configs.py (collect.sh)",
        "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = 1/2)",
        "key": "<op>_<layout>_<frame_len|imix>_<frames per launch>",
        "configs": {},
    }
    with open(os.path.join(dst, "pmc_configs.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["config", "kernel", "launches", "avg_FETCH_SIZE_KB", "avg_WRITE_SIZE_KB",
                    "hbm_bytes_per_launch", "avg_duration_ns"])
        for lab in sorted(acc):
            e = acc[lab]
            mean = lambda k: sum(e[k]) / len(e[k]) if e.get(k) else None  # noqa: E731
            fs, ws, du = mean("FETCH_SIZE"), mean("WRITE_SIZE"), mean("duration_ns")
            hbm = (2 * fs + (ws or 0)) * 1024 if fs is not None else None
            w.writerow([lab, names[lab], max(len(v) for v in e.values()), fs, ws, hbm, du])
            summary["configs"][lab] = {"kernel": names[lab], "fetch_size_kb": fs,
                                       "write_size_kb": ws, "hbm_bytes_per_launch": hbm,
                                       "avg_duration_ns": du,
                                       "launches": max(len(v) for v in e.values())}
    json.dump(summary, open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w"), indent=1)
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
