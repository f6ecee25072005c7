set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st256.bin timeout -k 10 200 python3 tools/ha_plan_time.py > $O/st256.log 2>&1 &&
python3 tools/ha_stamps.py $O/st256.bin > $O/st256.txt && python3 tools/ha_stamps_blocks.py $O/st256.bin 2 > $O/st256_blocks.txt
