set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
MPGPU_LIB=$L/libmpgpu_noovl.so timeout -k 10 200 python3 tools/ha_lone.py > $O/lone_noovl.log 2>&1 && cat $O/lone_noovl.log &&
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st_ovl.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st_ovl.log 2>&1 &&
MPGPU_LIB=$L/libmpgpu_stampnoovl.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st_noovl.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st_noovl.log 2>&1 &&
python3 tools/ha_stamps_blocks.py $O/st_ovl.bin 4 > $O/st_ovl.txt && python3 tools/ha_stamps_blocks.py $O/st_noovl.bin 4 > $O/st_noovl.txt &&
timeout -k 10 300 python3 tools/mppi_libm_ab.py > $O/libm_fdlibm.log 2>&1 && cat $O/libm_fdlibm.log &&
MPGPU_LIB=$L/libmpgpu_ocml.so timeout -k 10 300 python3 tools/mppi_libm_ab.py > $O/libm_ocml.log 2>&1 && cat $O/libm_ocml.log
