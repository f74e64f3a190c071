#!/bin/bash
# Small-shape likelihood launches (likelihood_other_configs) at the default tasks per CU and at
# fixed values (context option lik_tasks_per_cu), two alternated rounds on one box.
mkdir -p gpurun_out/abl
for r in 1 2; do
  for t in 0 2 3 4; do
    opt=""; [ $t != 0 ] && opt="--option lik_tasks_per_cu=$t"
    timeout -k 10 200 python bench.py --steps 20 --warmup 4 --cpu-seconds 0 --mh-steps 0 --src-steps 0 --source-lik-steps 0 $opt > gpurun_out/abl/t$t.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); o=d['likelihood_other_configs']; print('t=$t', {k.split('_')[0]: round(v['launch_us'],1) for k,v in o.items()}, 'cfg5', round(d['ms_per_step']*1000,1))" gpurun_out/abl/t$t.json
  done
done
