import csv,glob,collections,sys
for v in sys.argv[1].split():
    for cfg in ["cfg2_1m_sh3_1080p_f16","cfg3_5m_sh3_4k_f16"]:
        fs=glob.glob(f"gpurun_out/ab/kt_{v}_{cfg}/**/*kernel_trace.csv",recursive=True)
        if not fs: continue
        rows=list(csv.DictReader(open(fs[0])))
        rows.sort(key=lambda r:int(r['Start_Timestamp']))
        seq=collections.defaultdict(list)
        idx=collections.Counter()
        for r in rows:
            n=r['Kernel_Name'].split('(')[0].replace('void ','').replace('gsm::','')
            if n.startswith('k_project'): idx=collections.Counter()
            idx[n]+=1
            seq[f"{n}#{idx[n]}"].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
        tot=0; out=[]
        for k,vals in seq.items():
            if len(vals)>10 and ('radix' in k or 'tile' in k):
                vals=vals[3:]; m=sum(vals)/len(vals); tot+=m
                out.append(f"{k.split('<')[0].replace('k_radix_','')}={m:.1f}")
        print(v,cfg[:4]," ".join(out), f"TOTAL={tot:.1f}")
