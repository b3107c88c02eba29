"""Per-kernel PMC summary for the prefill kernels (tools/pmc_prefill.sh output).
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the counter sums matrix-core busy cycles
over all SIMDs (32 per 32x32x16 MFMA, MI355X_MICROARCH.md PMC units) and GRBM_GUI_ACTIVE sums the 8 XCDs' clocks.
SQ_WAIT_* / SQ_ACTIVE_* / SQ_WAVE_CYCLES are quad-cycles; ratios among them are reported as is.
usage: python tools/pmc_prefill_summary.py DIR [--json OUT]"""
import collections
import csv
import glob
import json
import sys

KERNELS = ["k_gemm_q6p", "k_gemm_q4v4", "k_gemm_q4v3", "k_gemm_q6v3", "k_gemm_kq", "k_gemm_q80s2", "k_fa_prefill_mfma3", "k_fa_prefill_mfma2", "k_fa_prefill_mfma",
           "k_act_frag3", "k_act_frag6", "k_splitk_reduce"]


def short(name):
    base = name.split("(")[0].replace("void ", "")
    for k in KERNELS:
        if base.startswith(k):
            return base[:90]
        if base.startswith("_Z") and k in base:      # mangled (vector-typed args): k + template args
            t = base.split(k, 1)[1]
            return k + ("<" + ",".join(__import__("re").findall(r"Li(\d+)E", t.split("EEv")[0])) + ">" if t.startswith("I") else "")
    return None


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(d + "/p*/**/pmc_counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    for f in glob.glob(d + "/trace/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    out = {}
    for k, cs in sorted(acc.items()):
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"dispatches": max(len(v) for v in cs.values()), "counters_avg": {c: round(x, 1) for c, x in sorted(a.items())}}
        if k in dur:
            e["trace_avg_us"] = round(sum(dur[k]) / len(dur[k]), 2)
        g = a.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            # time-weighted over the kernel's dispatches (sums of both counters, same passes' dispatch sets)
            e["mfma_busy_frac"] = round(sum(cs["SQ_VALU_MFMA_BUSY_CYCLES"]) / (sum(cs["GRBM_GUI_ACTIVE"]) / 8 * 1024), 4)
            if k in dur:
                e["clock_ghz_est"] = round(g / 8 / (e["trace_avg_us"] * 1e3), 3)
        if "SQ_WAVE_CYCLES" in a:
            wc = a["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in a:
                    e[c.lower().replace("sq_", "") + "_per_wave_cycle"] = round(a[c] / wc, 4)
        if "SQ_LDS_BANK_CONFLICT" in a and a.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_per_active"] = round(a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"], 4)
        out[k] = e
        print(k, json.dumps({x: y for x, y in e.items() if x != "counters_avg"}))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
