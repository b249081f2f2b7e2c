import csv, collections, re, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def key(n):
    if 'put_sync' in n: return 'sync'
    if 'copy2d' in n: return 'copy'
    m=re.search(r'(hx_kernel|vkernel)<([^>]*)>', n)
    return (m.group(1)+'<'+m.group(2)+'>') if m else n[:40]
seq=[(key(r['Kernel_Name']), int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows]
# per stencil kind: collect cycles stencil -> next stencil of the same kind
stats=collections.defaultdict(lambda: collections.defaultdict(list))
for i in range(len(seq)-1):
    k,s,e=seq[i]
    if k in ('sync','copy') or 'FillFunctor' in k: continue
    # following non-stencil kernels until next stencil
    j=i+1; parts=[]
    while j<len(seq) and seq[j][0] in ('sync','copy'):
        parts.append(seq[j]); j+=1
    if j>=len(seq) or seq[j][0]!=k: continue
    nxt=seq[j]
    st=stats[k+' + '+'+'.join(p[0] for p in parts)]
    st['stencil'].append((e-s)/1e3)
    prev=e
    for n,(pk,ps,pe) in enumerate(parts):
        st[f'gap{n}'].append((ps-prev)/1e3); st[f'{pk}{n}'].append((pe-ps)/1e3); prev=pe
    st['gap_next'].append((nxt[1]-prev)/1e3)
    st['cycle'].append((nxt[1]-s)/1e3)
for k,st in stats.items():
    n=len(st['cycle'])
    if n<20: continue
    med=lambda v: sorted(v)[len(v)//2]
    print(f"{k}  n={n}")
    print('   '+'  '.join(f"{a}={med(v):.2f}" for a,v in st.items()))
