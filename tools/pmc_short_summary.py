"""Summary of tools/pmc_short.sh: per case, the mat-vec kernel's memory-side bytes per launch (FETCH_SIZE x 2 per the
gfx950 correction of MI355X_MICROARCH.md "HBM", + WRITE_SIZE; KB -> B), its rocprofv3 average duration, the
algorithmic bytes (weights + activation) and the resulting fraction of the 8 TB/s HBM peak.
usage: python tools/pmc_short_summary.py OUTDIR > profiles/TAG_short_matvec_pmc.json"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
E, F = 4096, 14336
ALG = {  # case -> algorithmic bytes per launch (weight rows + Q8_K / f32 activation read + outputs written)
    "rs wo q4k pro0": E * E // 256 * 144 + (E + E // 256 * 4 + E // 16 * 2) + E * 4,
    "rs qkv q4k pro1 rope": (E + 2048) * E // 256 * 144 + E * 4 + (E + 2048) * 2,
    "rs down q4k pro2": E * F // 256 * 144 + F * 4 + E * 4,
    "rs down q6k pro2": E * F // 256 * 210 + F * 4 + E * 4,
}
out = {"source": "tools/pmc_short.sh (tools/stream_probe.py dec: weights rotated past the Infinity Cache, 40 timed "
                  "launches + warm-ups per case)", "hbm_peak_GBps": 8000.0, "cases": {}}
for cdir in sorted(glob.glob(os.path.join(d, "c*"))):
    case = open(os.path.join(cdir, "case.txt")).read().strip()

    def avg(sub, ctr):
        v = []
        for f in glob.glob(os.path.join(cdir, sub, "**", "pmc_counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "gemv" in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                    v.append(float(r["Counter_Value"]))
        return sum(v) / len(v) if v else None
    fe, wr = avg("FETCH_SIZE", "FETCH_SIZE"), avg("WRITE_SIZE", "WRITE_SIZE")
    dur = None
    for f in glob.glob(os.path.join(cdir, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemv" in r["Name"]:
                dur = float(r["AverageNs"]) / 1e3
    alg = ALG.get(case)
    rec = {"algorithmic_bytes": alg, "avg_us": dur}
    if fe is not None and wr is not None:
        rec["traffic_bytes_per_launch"] = round(2 * fe * 1024 + wr * 1024)
        if alg:
            rec["traffic_over_algorithmic"] = round(rec["traffic_bytes_per_launch"] / alg, 3)
    if dur and alg:
        rec["achieved_GBps"] = round(alg / (dur * 1e-6) / 1e9, 1)
        rec["frac_of_peak"] = round(rec["achieved_GBps"] / 8000.0, 4)
    out["cases"][case] = rec
print(json.dumps(out, indent=1))
