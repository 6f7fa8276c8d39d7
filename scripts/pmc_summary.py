"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) per kernel.

    python scripts/pmc_summary.py gpurun_out/pmc [--json profiles/pmc_r01.json]

Per kernel: mean dispatch duration and per-dispatch means of every counter collected, plus
derived ratios.  HBM bytes follow MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are KiB, and
on gfx950 FETCH_SIZE reports half the bytes of a wide streaming read, so it is doubled.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def family(name):
    m = re.search(r"hd::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def load(root):
    acc = defaultdict(lambda: defaultdict(float))        # kernel -> counter -> sum
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for f in glob.glob(os.path.join(root, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            key = (f, r["Dispatch_Id"])
            disp[(k, r["Counter_Name"])].add(key)
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    out = {}
    for k, cs in acc.items():
        row = {"dispatch_ms": sum(dur[k].values()) / max(len(dur[k]), 1)}
        for c, v in cs.items():
            row[c] = v / max(len(disp[(k, c)]), 1)
        out[k] = row
    return out


def derive(row):
    d = {}
    if row.get("SQ_WAVE_CYCLES"):
        d["valu_active_per_wave_cycle"] = row.get("SQ_ACTIVE_INST_VALU", 0) / row["SQ_WAVE_CYCLES"]
    if row.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict_share"] = row.get("SQ_LDS_BANK_CONFLICT", 0) / row["SQ_LDS_IDX_ACTIVE"]
    if "FETCH_SIZE" in row:
        d["hbm_read_bytes"] = 2.0 * row["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in row:
        d["hbm_write_bytes"] = row["WRITE_SIZE"] * 1024.0
    if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
        d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = load(a.root)
    fam = {}
    for k, r in sorted(rows.items(), key=lambda kv: -kv[1]["dispatch_ms"]):
        d = derive(r)
        print("%s\n  dispatch %.3f ms" % (k[:100], r["dispatch_ms"]))
        for c in sorted(r):
            if c != "dispatch_ms":
                print("  %-28s %.4g" % (c, r[c]))
        for c in sorted(d):
            print("  %-28s %.4g" % ("= " + c, d[c]))
        if "hbm_bytes" in d:
            fam.setdefault(family(k), []).append(d["hbm_bytes"])
    if a.json:
        per_launch = {f: sum(v) / len(v) for f, v in fam.items()}
        for pre in ("k_stage1", "k_stage2"):       # the families bench.py reports
            vals = [b for f, v in fam.items() if f.startswith(pre) for b in v]
            if vals:
                per_launch[pre] = sum(vals) / len(vals)
        json.dump({"source": a.root,
                   "note": "HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B), mean over the "
                           "instantiations of a kernel family (gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md)",
                   "hbm_bytes_per_launch": per_launch}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
