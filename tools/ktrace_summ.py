import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = max(i for i, r in enumerate(rows) if 'spin_kernel' in r['Kernel_Name'])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[idx + 1:]:
    k = r['Kernel_Name'].split('(')[0][:100]
    agg[k][0] += 1
    agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
reps = int(sys.argv[2])
tot = sum(v[1] for v in agg.values()) / reps
print(f"TOTAL kernel ms per forward {tot:.2f}, kernels per forward {sum(v[0] for v in agg.values())/reps:.0f}")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{t/reps:9.2f} ms {c/reps:7.1f}  {k}")
