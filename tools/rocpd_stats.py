"""Per-kernel summary (the rocprofv3 --stats kernel table) from a rocprofv3 rocpd database (ROCm 7 writes
<out>_results.db when no --output-format is given).  Usage: python3 tools/rocpd_stats.py run_results.db [csv_out]"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                      "max(vgpr_count), max(accum_vgpr_count), max(lds_size), max(grid_x), max(workgroup_x) "
                      "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage", "VGPR", "AGPR", "LDS",
           "GridX", "WGX"]
    out = [[r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100.0 * r[2] / total, 2), r[6], r[7], r[8], r[9], r[10]]
           for r in rows]
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            w.writerows(out)
    for r in out[:30]:
        print("%-72s %6d %9.2f us %6.2f%%  vgpr %s lds %s grid %s" % (r[0][:72], r[1], r[3] / 1e3, r[6], r[7], r[9], r[10]))


if __name__ == "__main__":
    main()
