"""Summarise a scripts/gpu_prof.sh run: per-kernel avg duration (trace) and per-launch counters."""
import csv, sys, collections, json, os
d = sys.argv[1]
def short(n):
    n = n.split('(')[0]
    return n.replace('void ', '').replace('tt2::', '')
st = {}
for r in csv.DictReader(open(os.path.join(d, 'trace', 'run_kernel_stats.csv'))):
    st[short(r['Name'])] = (int(r['Calls']), float(r['AverageNs']) / 1e3, float(r['Percentage']))
ctr = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ('fetch', 'write', 'tcc', 'sq'):
    p = os.path.join(d, sub, 'run_counter_collection.csv')
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        ctr[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
print('%-28s %6s %9s %6s %12s %12s %8s %10s' % ('kernel', 'calls', 'avg_us', 'pct', 'FETCH_KB', 'WRITE_KB', 'L2hit%', 'clk_GHz'))
out = {}
for k, (c, us, pct) in sorted(st.items(), key=lambda x: -x[1][0] * x[1][1]):
    cc = ctr.get(k, {})
    avg = lambda n: sum(cc[n]) / len(cc[n]) if n in cc and cc[n] else float('nan')
    f, w = avg('FETCH_SIZE'), avg('WRITE_SIZE')
    h, m = avg('TCC_HIT_sum'), avg('TCC_MISS_sum')
    g = avg('GRBM_GUI_ACTIVE')
    hit = 100 * h / (h + m) if h == h and (h + m) > 0 else float('nan')
    clk = g / 8 / (us * 1e3) if g == g else float('nan')
    print('%-28s %6d %9.2f %6.2f %12.1f %12.1f %8.1f %10.2f' % (k[:28], c, us, pct, f, w, hit, clk))
    out[k] = dict(calls=c, avg_us=us, fetch_kb=f, write_kb=w, l2_hit_pct=hit,
                  hbm_bytes_per_launch=(2 * f + w) * 1024 if f == f and w == w else None)
json.dump(out, open(os.path.join(d, 'summary.json'), 'w'), indent=1)
