import csv, collections, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + '/pmc*/p_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('klf::(anonymous namespace)::', '').replace('(klf::RunArgs)', '').replace('void ', '')
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    if not any(x in k for x in ('k_scan', 'k_scatter', 'k_tail', 'k_compact', 'k_count')): continue
    print(k, {c: '%.3g' % (sum(v) / len(v)) for c, v in sorted(d.items())})
