import json,sys
d=json.load(open(sys.argv[1] if len(sys.argv)>1 else 'gpurun_out/stamps.json'))
for k,v in d.items():
    if isinstance(v,dict):
        print(k, 'span %.2f skew %.2f gap %s waves %d'%(v['span_us'],v['start_skew_us'],v.get('gap_to_next_us'),v['waves']), {p:(round(x['median_us'],2),round(x['max_us'],2)) for p,x in v['phases'].items()}, {k2:(round(x['median_us'],2),round(x['max_us'],2),round(x['end_us'],2)) for k2,x in v.items() if k2.startswith('part_')})
    else: print(k,v)
