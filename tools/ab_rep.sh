mkdir -p gpurun_out/ab
for i in 1 2 3; do for v in default old; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 400 --warmup 40 --cpu-seconds 0 --mh-steps 0 --src-steps 0 --source-lik-steps 20 > gpurun_out/ab/${v}_$i.json || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['roofline']['launch_us'],2), round(d['likelihood_source_branch']['launch_us'],1))" gpurun_out/ab/${v}_$i.json
done; done
