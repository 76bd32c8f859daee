import json,sys
d0=sys.argv[1]
for i in sys.argv[2:]:
    for v in ('base','new'):
        for l in open(f'{d0}/{v}.{i}.jsonl'):
            if l.startswith('{'):
                d=json.loads(l); r=d['roofline']; c=d.get('channel_sharded',{}).get('resident',{})
                print(v,i,r['kernel_ms'],r['frac'],'| c5',c.get('ms_per_step'),c.get('roofline_frac_per_gpu'))
