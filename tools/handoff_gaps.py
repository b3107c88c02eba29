"""Reads a rocprofv3 --kernel-trace --hip-trace run of tools/handoff_trace.py (CSV) and prints, for the N-stage
decode steps, where each stage boundary's time goes: the last kernel of stage s, the hand-off kernels (copyBuffer),
the first kernel of stage s+1, per queue, plus the host-side HIP calls in between.

  python3 tools/handoff_gaps.py gpurun_out/.../ho_kernel_trace.csv [hip_api_trace.csv]"""
import csv
import sys
from collections import Counter, defaultdict


def main():
    kt = list(csv.DictReader(open(sys.argv[1])))
    for r in kt:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    kt.sort(key=lambda r: r["s"])
    # the last decode steps: graph kernels of the single-token step (k_gemv_rs / k_fa_*) on several queues
    queues = Counter(r["Queue_Id"] for r in kt)
    print("dispatches per queue:", dict(queues))
    # find the argmax_final kernels (one per token, end of the last stage)
    ends = [r for r in kt if "argmax_final" in r["Kernel_Name"]]
    print("argmax_final count", len(ends))
    # take the last 8 tokens of the run
    last = ends[-9:]
    for a, b in zip(last, last[1:]):
        seg = [r for r in kt if a["e"] < r["s"] <= b["e"]]
        print("token: %.1f us, %d kernels" % ((b["e"] - a["e"]) / 1e3, len(seg)))
        prev = a
        t0 = a["e"]
        gaps = []
        for r in seg:
            gap = (r["s"] - prev["e"]) / 1e3
            if gap > 4 or "rocclr" in r["Kernel_Name"] or r["Queue_Id"] != prev["Queue_Id"]:
                gaps.append("  +%8.1f us gap %6.1f  q%s %s (%.1f us)" % ((r["s"] - t0) / 1e3, gap, r["Queue_Id"],
                                                                       r["Kernel_Name"][:60], (r["e"] - r["s"]) / 1e3))
            prev = r
        print("\n".join(gaps[:40]))
        break
    if len(sys.argv) > 2:
        ht = list(csv.DictReader(open(sys.argv[2])))
        cnt = Counter(r["Function"] for r in ht)
        dur = defaultdict(int)
        for r in ht:
            dur[r["Function"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print("host HIP calls (count, total us):")
        for f, c in cnt.most_common(25):
            print("  %-40s %7d %10.1f" % (f, c, dur[f] / 1e3))


if __name__ == "__main__":
    main()
