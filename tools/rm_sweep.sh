for rm in 6 0 6 0; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --render-mod $rm > gpurun_out/rm_$rm.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/rm_$rm.json')); print('render_mod $rm', round(d['ms_per_step'],4), {k:round(v*1e3,1) for k,v in d['stage_ms'].items() if k in ('preprocess','composite')})"
done
