set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_likelihood.py -k "planned or option or cut_by_lds or tape_replay" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_grp2.log 2>&1 || { tail -30 gpurun_out/pt_grp2.log; exit 1; }
tail -3 gpurun_out/pt_grp2.log
for g in 1 2 4; do
  echo "group $g"; timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets default,weights,p_zones --options "{\"mh_group\": $g}" 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
done
