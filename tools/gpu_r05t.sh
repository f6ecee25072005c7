# phase stamps of the 256-scenario plan with the full-width pipelined launch
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st.bin timeout -k 10 200 python3 tools/ha_plan_time.py > $O/st.log 2>&1 &&
python3 tools/ha_stamps_wide.py $O/st.bin > $O/wide.txt && cat $O/wide.txt &&
python3 tools/ha_stamps_blocks.py $O/st.bin 12 > $O/st.txt && rm -f $O/st.bin
