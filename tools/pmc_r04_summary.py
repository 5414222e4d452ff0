#!/usr/bin/env python3
"""Summarise a tools/pmc_r04.sh run (gpurun_out/pmc_r04) into profiles/<tag>_asm_counters.json:

  * assembly value kernels (k_asm_tet4_acc<1> / <3>, 10M cube): SQ wave cycles / waits / VALU / LDS counters and
    HBM bytes (FETCH_SIZE x 2 x 1024 -- the gfx950 streaming-read correction of MI355X_MICROARCH.md -- plus
    WRITE_SIZE x 1024) of the last dispatch, against SURVEY 8(d)'s B_asm = 112 M + 8 nnz (x bs^2);
  * BASELINE configs[4] (tools/bench_mixed.py): per kernel name the average duration (trace pass) and the HBM bytes
    of its last dispatch (FETCH / WRITE passes) -- k_iso_ke and the stored-K_e assembly kernels.

    python tools/pmc_r04_summary.py --tag r04b [--dir gpurun_out/pmc_r04]
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M10, NNZ10 = 10_110_954, 25_575_838   # the 10M cube: tets, node-graph nonzeros


def last_dispatch(path, sub):
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    if not rows:
        return {}, None
    last = max(int(r["Dispatch_Id"]) for r in rows)
    agg = {}
    name = None
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            name = r["Kernel_Name"]
    return agg, name


def hbm(fetch_kb, write_kb):
    return 2 * 1024 * fetch_kb + 1024 * write_kb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out", "pmc_r04"))
    a = ap.parse_args()
    out = {"source": "tools/pmc_r04.sh (one rocprofv3 --pmc pass per counter set)", "assembly": {}, "mixed": {}}
    for kind, bs in (("poisson", 1), ("elastic", 3)):
        d = os.path.join(a.dir, f"asm_{kind}")
        sq, name = last_dispatch(d + "_sq/run_counter_collection.csv", "k_asm_tet4_acc")
        fe, _ = last_dispatch(d + "_fetch/run_counter_collection.csv", "k_asm_tet4_acc")
        wr, _ = last_dispatch(d + "_write/run_counter_collection.csv", "k_asm_tet4_acc")
        b_asm = 112 * M10 + 8 * NNZ10 * bs * bs
        t = hbm(fe.get("FETCH_SIZE", 0.0), wr.get("WRITE_SIZE", 0.0))
        e = {"kernel": name, "counters": sq, "FETCH_SIZE_KB": fe.get("FETCH_SIZE"), "WRITE_SIZE_KB": wr.get("WRITE_SIZE"),
             "hbm_bytes": t, "B_asm": b_asm, "traffic_over_B_asm": t / b_asm if b_asm else None}
        if sq.get("SQ_WAVE_CYCLES"):
            e["wait_share"] = sq.get("SQ_WAIT_ANY", 0.0) / sq["SQ_WAVE_CYCLES"]
        out["assembly"][kind] = e
    stats = os.path.join(a.dir, "mixed_trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        fe_p = os.path.join(a.dir, "mixed_fetch", "run_counter_collection.csv")
        wr_p = os.path.join(a.dir, "mixed_write", "run_counter_collection.csv")
        for r in csv.DictReader(open(stats)):
            n = r["Name"]
            if not any(k in n for k in ("k_iso_ke", "k_assemble_ke", "k_csr_add_sell", "k_tet4_ke", "k_graph",
                                        "k_inc_l", "k_sell_fill_graph")):
                continue
            key = n.split("(")[0]
            fe, _ = last_dispatch(fe_p, key) if os.path.exists(fe_p) else ({}, None)
            wr, _ = last_dispatch(wr_p, key) if os.path.exists(wr_p) else ({}, None)
            out["mixed"][key] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                 "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                 "last_dispatch_hbm_bytes": hbm(fe.get("FETCH_SIZE", 0.0), wr.get("WRITE_SIZE", 0.0)),
                                 "FETCH_SIZE_KB": fe.get("FETCH_SIZE"), "WRITE_SIZE_KB": wr.get("WRITE_SIZE")}
    p = os.path.join(ROOT, "profiles", f"{a.tag}_asm_counters.json")
    json.dump(out, open(p, "w"), indent=1)
    print(p)


if __name__ == "__main__":
    main()
