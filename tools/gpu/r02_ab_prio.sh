mkdir -p gpurun_out/prio
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/prio/base$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_prio.so bench.py --no-cpu-baseline --steps 30 > gpurun_out/prio/prio$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; a=json.load(open('gpurun_out/prio/base$rep.json')); b=json.load(open('gpurun_out/prio/prio$rep.json'))
print('rep $rep base', a['roofline']['kernel_ms'], a['roofline']['frac'], '| prio', b['roofline']['kernel_ms'], b['roofline']['frac'])"
done
