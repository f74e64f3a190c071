#!/bin/bash
# Round-5 PMC passes of the mixture sampler (mh_kernel, cfg5, 256 chains): the bench's sampler leg
# alone, 3000 timed steps, no burn-in (tools/pmc.sh passes; summary in gpurun_out/pmc_mh/pmc.json).
PMC_OUT=gpurun_out/pmc_mh timeout -k 10 900 bash tools/pmc.sh --steps 2 --warmup 1 --mh-steps 3000 --mh-burnin 0 --src-steps 0 --source-lik-steps 0 --other-steps 0 --cpu-sampler-seconds 0 --src-sampler-steps 0 > gpurun_out/pmc_mh.log 2>&1 || { tail -20 gpurun_out/pmc_mh.log; exit 1; }
tail -6 gpurun_out/pmc_mh.log
