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


def short(name):
    """'void hd::k_stage2_pair<5, 3, 2>(hd::Stage2Args, int const*)' -> 'k_stage2_pair<5, 3, 2>'
    (the name hd_plan_kernel reports)."""
    s = re.sub(r"^void ", "", name.strip())
    s = re.sub(r"^hd::", "", s)
    depth, out = 0, []
    for ch in s:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)


_DISP = defaultdict(set)                                   # (kernel, counter) -> dispatches


def load(root):
    acc = defaultdict(lambda: defaultdict(float))        # kernel -> counter -> sum
    disp = _DISP
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
    ap.add_argument("--commit", default="")
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
        kernels = {}
        for k, r in rows.items():
            d = derive(r)
            if "hbm_bytes" not in d:
                continue
            e = {"launches": len(next(iter(v for kk, v in _DISP.items() if kk[0] == k), [])) or None,
                 "dispatch_ms": r["dispatch_ms"]}
            e.update({c: d[c] for c in ("hbm_read_bytes", "hbm_write_bytes", "hbm_bytes") if c in d})
            for c in ("valu_active_per_wave_cycle", "lds_conflict_share"):
                if c in d:
                    e[c] = d[c]
            kernels[short(k)] = e
        json.dump({"source": a.root, "commit": a.commit,
                   "note": "per launch, mean over the kernel's dispatches in the profiled run: hbm_bytes = "
                           "2*FETCH_SIZE + WRITE_SIZE (KiB -> B; gfx950 FETCH_SIZE counts half of a wide "
                           "streaming read, MI355X_MICROARCH.md); keys are the exact kernel names "
                           "(hd_plan_kernel), so bench.py only takes a traffic figure for the kernel it times",
                   "kernels": kernels}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
