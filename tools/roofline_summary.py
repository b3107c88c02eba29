"""Summarize tools/profile_round.sh output into profiles/TAG_*:
  TAG_roofline_pmc.json   -- per-launch HBM traffic of the roofline kernel (FETCH_SIZE x 2 per the
                             gfx950 correction in MI355X_MICROARCH.md "HBM", + WRITE_SIZE; KB -> B)
                             and its rocprofv3 average duration, next to bench.py's HIP-event figure
  TAG_roofline_kernel_stats.csv, TAG_bench_kernel_stats.csv -- rocprofv3 --stats summaries
usage: python tools/roofline_summary.py TAG [KERNEL_SUBSTRING]"""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "k_gemv_rs"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "gpurun_out", "prof_" + tag)


def counter(name):
    vals = []
    for f in glob.glob(os.path.join(out, name.lower().split("_")[0], "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals, None


fetch, _ = counter("FETCH_SIZE")
write, _ = counter("WRITE_SIZE")
durs, kname = [], None
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            kname = r["Kernel_Name"]
bench_line = None
for line in open(os.path.join(out, "trace.log")):
    if line.startswith("{"):
        bench_line = json.loads(line)
res = {
    "kernel": kname,
    "launches": {"fetch": len(fetch), "write": len(write), "trace": len(durs)},
    "fetch_size_kb_avg": sum(fetch) / len(fetch),
    "write_size_kb_avg": sum(write) / len(write),
    "traffic_bytes_per_launch": round(2 * sum(fetch) / len(fetch) * 1024 + sum(write) / len(write) * 1024),
    "rocprof_avg_us": round(sum(durs) / len(durs) / 1e3, 3),
    "bench_hip_event_avg_us": bench_line["roofline"]["avg_us"] if bench_line else None,
    "algorithmic_bytes_per_launch": bench_line["roofline"]["bytes_per_launch"] if bench_line else None,
    "note": "FETCH_SIZE doubled (gfx950: half the bytes of wide coalesced reads); includes the warm-up launches; "
            "8 weight pairs (504 MiB) rotated so the 256 MiB Infinity Cache cannot serve repeats",
}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
with open(os.path.join(root, "profiles", tag + "_roofline_pmc.json"), "w") as f:
    json.dump(res, f, indent=1)


def fa_summary():
    """decode attention (k_fa_dec4 + k_fa_comb4, tools/fa_dec_bench.py variant 3 at 3850 cached keys): per kernel
    the memory-side bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE) and the rocprofv3 average duration"""
    def per_kernel(d, cname):
        acc = {}
        for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                for kk in ("k_fa_dec4", "k_fa_comb4"):
                    if kk in r["Kernel_Name"] and r["Counter_Name"] == cname:
                        acc.setdefault(kk, []).append(float(r["Counter_Value"]))
        return {k: sum(v) / len(v) for k, v in acc.items()}
    fe, wr = per_kernel("fa_fetch", "FETCH_SIZE"), per_kernel("fa_write", "WRITE_SIZE")
    du = {}
    for f in glob.glob(os.path.join(out, "fa_trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for kk in ("k_fa_dec4", "k_fa_comb4"):
                if kk in r["Kernel_Name"]:
                    du.setdefault(kk, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    kv_bytes = 2 * 8 * 128 * 2 * 3851
    out_fa = {"workload": "Llama-3-8B decode attention, 3850 cached keys, 32 q / 8 kv heads x 128, f16 KV, "
                          "32 layers' caches rotated (tools/fa_dec_bench.py, variant 3)",
              "algorithmic_bytes_k_fa_dec4": kv_bytes + 32 * 128 * 2 + 32 * 32 * 130 * 4,
              "note": "FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md HBM); KB -> B"}
    for kk in ("k_fa_dec4", "k_fa_comb4"):
        if kk in fe and kk in wr:
            out_fa[kk] = {"traffic_bytes_per_launch": round(2 * fe[kk] * 1024 + wr[kk] * 1024),
                          "fetch_size_kb_avg": fe[kk], "write_size_kb_avg": wr[kk],
                          "rocprof_avg_us": round(sum(du.get(kk, [0])) / max(1, len(du.get(kk, []))) / 1e3, 3)}
    with open(os.path.join(root, "profiles", tag + "_fa_pmc.json"), "w") as f:
        json.dump(out_fa, f, indent=1)
    for f in glob.glob(os.path.join(out, "fa_trace", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(root, "profiles", "%s_fa_kernel_stats.csv" % tag))
    print(json.dumps(out_fa, indent=1))


if os.path.isdir(os.path.join(out, "fa_fetch")):
    fa_summary()
for src, dst in (("trace", "roofline"), ("bench", "bench")):
    for f in glob.glob(os.path.join(out, src, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(root, "profiles", "%s_%s_kernel_stats.csv" % (tag, dst)))
print(json.dumps(res, indent=1))
