import csv, collections, sys
def load(path):
    rows = list(csv.DictReader(open(path)))
    d = collections.OrderedDict()
    for r in rows:
        n = r['Kernel_Name']
        if 'hx_kernel' not in n and 'vkernel' not in n: continue
        k = int(r['Dispatch_Id'])
        e = d.setdefault(k, {'name': n[n.find('<'):n.find('>')+1], 'vgpr': r['VGPR_Count']})
        e[r['Counter_Name']] = e.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    return d
for p in sys.argv[1:]:
    d = load(p)
    print(p, len(d))
    for k, e in d.items():
        print(k, e['name'][:60], {c: round(v/1e6, 3) for c, v in e.items() if c not in ('name','vgpr')})
