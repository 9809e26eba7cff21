import csv, collections, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('hgsr::', '')
        agg[name][r['Counter_Name']].append(float(r['Counter_Value']))
        meta[name] = (r['VGPR_Count'], r['Accum_VGPR_Count'], r['SGPR_Count'], r['LDS_Block_Size'])
for k, d in agg.items():
    print(k, 'vgpr/agpr/sgpr/lds', meta[k])
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.4g}")
