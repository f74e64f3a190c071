set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
rm -f gpurun_out/ab_*
BENCH_ARGS="--mh-steps 0" STEPS=300 bash tools/ab.sh default:SBZ_LIK_KERNEL=zoned || exit 1
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for k in dense ws; do
  SBZ_LIK_KERNEL=$k timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc2/$k -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 --mh-steps 0 > gpurun_out/pmc2/$k.log 2>&1 || { echo "pmc $k failed"; tail -5 gpurun_out/pmc2/$k.log; exit 1; }
done
