"""Average PMC counter values per kernel-name prefix from rocprofv3 --pmc csv passes.
usage: python tools/pmc_summary.py DIR [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "gemv"
acc = collections.defaultdict(list)
for f in sorted(glob.glob(d + "/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            acc[(r["Kernel_Name"].split("(")[0][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("%-40s %-28s n=%3d avg=%14.1f" % (k, c, len(v), sum(v) / len(v)))
