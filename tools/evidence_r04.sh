set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "== $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
tail -c 300 gpurun_out/bench_default.json
rm -rf gpurun_out/prof4
run timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/prof4.log 2>&1
find gpurun_out/prof4 -name "*kernel_stats.csv" -exec head -12 {} \;
PMC_OUT=gpurun_out/pmc4 run timeout -k 10 900 bash tools/pmc.sh --mh-steps 0 --src-steps 0 --other-steps 0 > gpurun_out/pmc4.log 2>&1
tail -60 gpurun_out/pmc4.log
echo EV_OK
