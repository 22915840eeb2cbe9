import json,sys,glob
for f in sys.argv[1:]:
    for ln in open(f):
        if ln.startswith("{"):
            d=json.loads(ln); r=d["roofline"]
            print(f.split('/')[-1], round(d["value"]/1e9,3), "G", round(d["ms_per_step"]*1e3,1),"us", r["kernel"], "frac",round(r["frac"],3), "busy",round((r.get("avg_launch_busy_profiled_ms") or 0)*1e3,1), {k:round(v["busy_ms_per_step"]*1e3,1) for k,v in r["kernels"].items()})
