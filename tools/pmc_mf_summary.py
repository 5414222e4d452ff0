#!/usr/bin/env python3
"""Per-kernel summary of a tools/pmc_mf.sh run: average duration (trace pass), and of each kernel's last dispatch the
SQ counters, HBM bytes (FETCH_SIZE x 2 x 1024, the gfx950 streaming-read correction, + WRITE_SIZE x 1024).

    python tools/pmc_mf_summary.py [--dir gpurun_out/pmc_mf] [--match mf_] [--out file.json]
"""
import argparse
import csv
import glob
import json
import os


def stats(d):
    out = {}
    for p in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(p)):
            out[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def counters(d, sub):
    agg = {}
    for p in glob.glob(os.path.join(d, sub, "*counter_collection.csv")):
        rows = list(csv.DictReader(open(p)))
        last = {}
        for r in rows:
            last[r["Kernel_Name"]] = max(last.get(r["Kernel_Name"], -1), int(r["Dispatch_Id"]))
        for r in rows:
            if int(r["Dispatch_Id"]) == last[r["Kernel_Name"]]:
                k = agg.setdefault(r["Kernel_Name"], {})
                k[r["Counter_Name"]] = k.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="gpurun_out/pmc_mf")
    ap.add_argument("--match", default="")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    st = stats(a.dir)
    sq, fe, wr = counters(a.dir, "sq"), counters(a.dir, "fetch"), counters(a.dir, "write")
    res = {}
    for name, s in sorted(st.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]):
        if a.match not in name:
            continue
        e = dict(s)
        e.update(sq.get(name, {}))
        if name in fe and name in wr:
            e["hbm_bytes"] = 2 * 1024 * fe[name].get("FETCH_SIZE", 0) + 1024 * wr[name].get("WRITE_SIZE", 0)
            e["fetch_bytes_x2"] = 2 * 1024 * fe[name].get("FETCH_SIZE", 0)
            e["write_bytes"] = 1024 * wr[name].get("WRITE_SIZE", 0)
        if "SQ_WAVE_CYCLES" in e and e["SQ_WAVE_CYCLES"]:
            e["wait_share"] = e.get("SQ_WAIT_ANY", 0) / e["SQ_WAVE_CYCLES"]
        res[name] = e
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
