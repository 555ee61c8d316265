#!/usr/bin/env python3
"""Summarise a prof_round.sh output directory into profiles/-ready text.

Per kernel: calls and average duration (rocprofv3 --kernel-trace --stats),
and HBM bytes per dispatch from the PMC passes, corrected as
MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE tallies half the bytes of wide (16 B/lane)
coalesced streaming reads, so the read side is doubled.
Usage: summarize_prof.py <dir> [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split("(")[0].split("::")[-1].strip()


def kernel_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            out[k] = {"calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                      "avg_ms": float(r["AverageNs"]) / 1e6, "pct": float(r["Percentage"])}
    return out


def pmc(d, sub, counter):
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            acc[(short(r["Kernel_Name"]), r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in acc.items():
            per[k].append(v * 1024.0)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    d = sys.argv[1]
    ks = kernel_stats(d)
    fetch = pmc(d, "fetch", "FETCH_SIZE")
    write = pmc(d, "write", "WRITE_SIZE")
    sq = {}
    for sub in ("sq1", "sq2"):
        for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
            acc = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                acc[(short(r["Kernel_Name"]), r["Counter_Name"])] += float(r["Counter_Value"])
            for (k, c), v in acc.items():
                sq.setdefault(k, {})[c] = v
    rows = []
    for k in sorted(set(ks) | set(fetch) | set(write), key=lambda k: -ks.get(k, {}).get("total_ms", 0)):
        s = ks.get(k, {})
        f, w = fetch.get(k), write.get(k)
        hbm = (2 * f + w) if f is not None and w is not None else None
        rows.append({"kernel": k, **s, "fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_corrected": hbm})
    print("%-28s %6s %10s %10s %7s %14s %14s %14s" % ("kernel", "calls", "total_ms", "avg_ms", "pct",
                                                     "FETCH(raw)B", "WRITE B", "HBM B (2F+W)"))
    for r in rows:
        def g(x, fmt):
            return fmt % x if x is not None else "-"
        print("%-28s %6s %10s %10s %7s %14s %14s %14s" % (
            r["kernel"][:28], g(r.get("calls"), "%d"), g(r.get("total_ms"), "%.3f"), g(r.get("avg_ms"), "%.4f"),
            g(r.get("pct"), "%.2f"), g(r["fetch_bytes_raw"], "%.4g"), g(r["write_bytes"], "%.4g"),
            g(r["hbm_bytes_corrected"], "%.4g")))
    if sq:
        print("\nSQ counters (summed over dispatches of one build; quad-cycles for *_CYCLES/WAIT/ACTIVE):")
        for k, cs in sorted(sq.items()):
            print("  %-26s %s" % (k[:26], " ".join("%s=%.3g" % (c.replace("SQ_", ""), v) for c, v in sorted(cs.items()))))
    if "--json" in sys.argv:
        out = {"note": "per-launch HBM bytes from separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE in KiB; "
                       "FETCH doubled for gfx950 wide streaming reads per MI355X_MICROARCH.md)",
               "workload": json.load(open(os.path.join(d, "workload.json"))) if os.path.exists(
                   os.path.join(d, "workload.json")) else None,
               "kernels": {r["kernel"]: r for r in rows}}
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
