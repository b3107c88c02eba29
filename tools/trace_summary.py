"""Summarize a rocprofv3 kernel trace (decode region = after the last prefill-only kernel)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
ntok = int(sys.argv[2]) if len(sys.argv) > 2 else 20
last_pf = max((i for i, n in enumerate(names) if 'fa_prefill' in n or 'k_gemm' in n), default=-1)
dec = rows[last_pf + 1:]
d = collections.defaultdict(list)
for r in dec:
    d[r['Kernel_Name'].split('(')[0][:48]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = 0
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%-48s n=%5d avg=%7.2f us  per_token=%7.1f us" % (k, len(v), sum(v) / len(v), sum(v) / ntok))
    tot += sum(v) / ntok
t0 = int(dec[0]['Start_Timestamp']); t1 = int(dec[-1]['End_Timestamp'])
print('kernel sum per token %.1f us, wall per token %.1f us' % (tot, (t1 - t0) / 1e3 / ntok))
# launch boundaries: gap from the previous kernel's end to each kernel's start, per kernel name
gaps = collections.defaultdict(list)
for a, b in zip(dec, dec[1:]):
    gaps[b['Kernel_Name'].split('(')[0][:48]].append((int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3)
print('gaps before each kernel (us): ' + ', '.join('%s %.2f' % (k[:40], sum(v) / len(v)) for k, v in gaps.items()))
