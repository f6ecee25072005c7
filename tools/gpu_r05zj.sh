# per-block phase stamps of the persistent tail (lone 729-pop scenario): where its ~18.5 us per iteration go
set -o pipefail
O=gpurun_out/r05zj; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st.log 2>&1 &&
python3 tools/ha_stamps_blocks.py $O/st.bin 8 > $O/st.txt && rm -f $O/st.bin && head -60 $O/st.txt
