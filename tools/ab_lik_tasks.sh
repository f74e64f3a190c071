mkdir -p gpurun_out/abt
for t in 0 2 4 8 24; do
  OPT=""; [ $t = 0 ] || OPT="--option lik_tasks_per_cu=$t"
  SBZ_LIB_PATH=${SBZ_LIB_PATH:-} timeout -k 10 120 python bench.py $OPT --steps 20 --warmup 5 --cpu-seconds 0 --mh-steps 0 --src-steps 0 --source-lik-steps 0 --other-steps 200 > gpurun_out/abt/t$t.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); o=d['likelihood_other_configs']; print(sys.argv[1], round(d['roofline']['launch_us_event'],1), {k[:4]:round(v['launch_us'],1) for k,v in o.items() if k!='note'})" gpurun_out/abt/t$t.json
done
