"""Copy/kernel timeline of one pipelined host call from a rocprofv3
--kernel-trace --memory-copy-trace CSV pair: the key-cache kernels, the
key-grouping scatter and the H2D copies longer than 50 us, in us from the call's
first key-cache kernel.
Usage: python tools/copy_kernel_timeline.py <dir with run_*_trace.csv> <call index> <key-cache launches per call>"""
import csv,sys
d=sys.argv[1]; which=int(sys.argv[2]); per=int(sys.argv[3])
k=list(csv.DictReader(open(d+"/run_kernel_trace.csv")))
m=list(csv.DictReader(open(d+"/run_memory_copy_trace.csv")))
ev=[]
for r in k: ev.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),"K",r["Kernel_Name"].split("(")[0].replace("void ","").replace("nt::","")[:44],r.get("Stream_Id","")))
for r in m: ev.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),"M",r["Direction"][12:],r.get("Stream_Id","")))
ev.sort()
ks=[e for e in ev if e[2]=="K" and "keyset" in e[3]]
call=ks[which*per:(which+1)*per]
t0=call[0][0]-1_500_000; t1=call[-1][1]+100_000
for e in ev:
    if t0<=e[0]<=t1 and (e[2]=="M" and e[1]-e[0]>50_000 or "keyset" in e[3] or "scatter" in e[3]):
        print(f"{(e[0]-call[0][0])/1e3:9.1f} {(e[1]-call[0][0])/1e3:9.1f} {(e[1]-e[0])/1e3:8.1f} {e[2]} {e[3]} s{e[4]}")
