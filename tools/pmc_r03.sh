#!/bin/bash
# Round-3 PMC evidence: the source branch (repack_source_kernel + lik_source_rc_kernel, the bench's
# --mode source workload) and the sampler (mh_kernel, 256 chains x 3000 steps of the bench's
# sampler leg), each counter pass its own rocprofv3 run (tools/pmc.sh).
set -u
PMC_OUT=gpurun_out/pmc_src timeout -k 10 600 bash tools/pmc.sh --mode source --mh-steps 0 --src-steps 0 --source-lik-steps 0 > gpurun_out/pmc_src.log 2>&1 || { tail -20 gpurun_out/pmc_src.log; exit 1; }
tail -4 gpurun_out/pmc_src.log
PMC_OUT=gpurun_out/pmc_mh timeout -k 10 600 bash tools/pmc.sh --steps 2 --warmup 1 --mh-steps 3000 --mh-burnin 0 --src-steps 0 --source-lik-steps 0 > gpurun_out/pmc_mh.log 2>&1 || { tail -20 gpurun_out/pmc_mh.log; exit 1; }
tail -4 gpurun_out/pmc_mh.log
