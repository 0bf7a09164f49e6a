"""Per-kernel time of the LAST training step in a rocprofv3 kernel trace (the window between the last two
k_tr_adam launches): python scripts/train_step_kernels.py <run_kernel_trace.csv> [n]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
adam = [i for i, r in enumerate(rows) if 'k_tr_adam' in r['Kernel_Name']]
win = rows[adam[-2] + 1: adam[-1] + 1]
wall = (int(win[-1]['End_Timestamp']) - int(win[0]['Start_Timestamp'])) / 1e6
tot, cnt = collections.Counter(), collections.Counter()
for r in win:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('tt2::', '')
    tot[n] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    cnt[n] += 1
print('step window %.2f ms, kernel time %.2f ms, %d launches' % (wall, sum(tot.values()), len(win)))
for n, v in tot.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 25):
    print('%9.3f ms %5d  %s' % (v, cnt[n], n[:90]))
