import json,sys,glob,os
d0=sys.argv[1]
for f in sorted(glob.glob(d0+'/bench_*.jsonl')):
    for line in open(f):
        line=line.strip()
        if not line.startswith('{'): continue
        d=json.loads(line); st=d['stage_ms']
        print(os.path.basename(f), round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4), 'med', round(d['latency_ms_median'],4), 'dsort', round(st['depth_sort']*1e3,1), 'ranges', round(st['tile_ranges']*1e3,1), 'comp', round(st['composite']*1e3,1))
