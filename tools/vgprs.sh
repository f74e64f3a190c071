#!/bin/bash
# VGPR / spill counts of the likelihood kernels (cfg5 instantiations) for extra hipcc defines:
# tools/vgprs.sh [-DFOO=1 ...]
cd "$(dirname "$0")/../contact_zones_amd/csrc"
out=$(mktemp /tmp/vg.XXXX.s)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off "$@" -S --cuda-device-only sbz_lik.hip -o $out 2>/dev/null
for k in lik_mixture_kernelILi3ELi32ELi4ELb1ELb1E lik_mixture_kernelILi3ELi4ELi8ELb1ELb1E lik_source_rc_kernelILi3ELi32ELb1E lik_source_rc_kernelILi3ELi4ELb1E; do
  echo "$k $(grep -A20 "^\s*\.name:\s*_ZN3sbz.*${k}EEvNS_7LikArgsE" $out | grep -E "vgpr_count|vgpr_spill|sgpr_spill" | awk '{printf "%s %s  ", $1, $2}')"
done
rm -f $out
