set -o pipefail
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_stamp.so timeout -k 10 300 python -u tools/tb_stamps.py 100 p_zones 2>&1 | grep -v amdgpu.ids
