"""Summarise gpurun_out/pmc_cfg3 (tools/pmc_cfg3.sh) into profiles/<tag>_config3_pmc.json and the config-3 bench
kernel-trace stats into profiles/<tag>_config3_kernel_stats.csv.
FETCH_SIZE (KB) x 2 on gfx950 for wide streaming reads (MI355X_MICROARCH.md HBM section), WRITE_SIZE (KB) as is;
per launch of the k_q80t kernel, over the timed launches (8 weight copies rotated past the Infinity Cache).
usage: python3 tools/pmc_cfg3_summary.py [tag]"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.join(ROOT, "gpurun_out", "pmc_cfg3")
tag = sys.argv[1] if len(sys.argv) > 2 - 1 and len(sys.argv) > 1 else "r05"


def counters(path):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "k_q80t" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


out = {"source": "tools/pmc_cfg3.sh + tools/q80t_shapes.py (M = 32, 64 launches + 8 warm-up over 8 weight copies)",
       "peak_GBps": 8000.0, "achievable_GBps_guide": 6300.0, "shapes": {}}
for sh in ("qkv", "wo", "down", "gate_up"):
    t = json.load(open(os.path.join(D, "time_%s.json" % sh)))
    f, nf = counters(os.path.join(D, "fetch_" + sh))
    w, _ = counters(os.path.join(D, "write_" + sh))
    q, _ = counters(os.path.join(D, "sq_" + sh))
    fetch = 2 * f.get("FETCH_SIZE", 0.0) * 1024
    write = w.get("WRITE_SIZE", 0.0) * 1024
    rec = dict(t)
    rec.update({"fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
                "traffic_bytes_per_launch": round(fetch + write),
                "traffic_over_algo": round((fetch + write) / t["algo_bytes"], 3),
                "achieved_GBps": round(t["algo_bytes"] / t["us"] / 1e3, 1),
                "frac_of_peak": round(t["algo_bytes"] / t["us"] / 1e3 / 8000.0, 4),
                "launches_counted": nf.get("FETCH_SIZE", 0)})
    if q:
        wc = q.get("SQ_WAVE_CYCLES", 0.0)
        rec["sq"] = {k: round(v) for k, v in q.items()}
        if wc:
            rec["sq_frac"] = {"wait_any": round(q.get("SQ_WAIT_ANY", 0) / wc, 3),
                              "wait_inst_any": round(q.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                              "active_inst_any": round(q.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)}
    out["shapes"][sh] = rec
dst = os.path.join(ROOT, "profiles", "%s_config3_pmc.json" % tag)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
st = glob.glob(os.path.join(D, "trace", "*kernel_stats.csv"))
if st:
    shutil.copy(st[0], os.path.join(ROOT, "profiles", "%s_config3_kernel_stats.csv" % tag))
