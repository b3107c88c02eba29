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
            "4 weight pairs rotated so the 256 MiB Infinity Cache cannot serve repeats",
}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
with open(os.path.join(root, "profiles", tag + "_roofline_pmc.json"), "w") as f:
    json.dump(res, f, indent=1)
for src, dst in (("trace", "roofline"), ("bench", "bench")):
    for f in glob.glob(os.path.join(out, src, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(root, "profiles", "%s_%s_kernel_stats.csv" % (tag, dst)))
print(json.dumps(res, indent=1))
