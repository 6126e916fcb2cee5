#!/usr/bin/env python3
"""Per-kernel VGPRs / spills / occupancy from hipcc's kernel-resource-usage remarks.

    hipcc ... -Rpass-analysis=kernel-resource-usage 2> remarks.txt
    python tools/resusage.py remarks.txt [substring]
"""
import re
import subprocess
import sys


def parse(text):
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line) or re.search(r"Name: (\S+)", line)
        if m and "Function Name" in line or (m and "remark: Name" not in line and "Name:" in line
                                             and "Function" in line):
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"),
                         ("vspill", r"VGPRs Spill: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                         ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
        return out.stdout.splitlines()
    except Exception:
        return names


def main():
    text = open(sys.argv[1]).read()
    rows = parse(text)
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        if flt and flt not in n:
            continue
        n = re.sub(r"\(.*\)$", "", n)
        print(f"{r.get('vgpr', '?'):>4} vgpr {r.get('vspill', '?'):>3} spill occ {r.get('occ', '?')}"
              f" lds {r.get('lds', '?'):>6}  {n}")


if __name__ == "__main__":
    main()
