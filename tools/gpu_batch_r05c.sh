set -o pipefail
: > gpurun_out/r05_tb_stamps6.txt
for set in p_zones p_global; do SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_stamp.so timeout -k 10 300 python -u tools/tb_stamps.py 100 $set 2>&1 | grep -v amdgpu.ids >> gpurun_out/r05_tb_stamps6.txt || exit 1; done
cat gpurun_out/r05_tb_stamps6.txt
