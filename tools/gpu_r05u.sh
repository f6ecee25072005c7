# full-width winners' (t, u, v) (MPGPU_HA_FULL_TUV), the live-count mirror (MPGPU_HA_MIRROR), the full-width
# pipe (MPGPU_HA_FPIPE_BLOCKS): bit-exactness, timing, and the phase stamps of the 256-scenario plan
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_FULL_TUV=1" "MPGPU_HA_FULL_TUV=0" "MPGPU_HA_MIRROR=0" "MPGPU_HA_FPIPE_BLOCKS=0" "MPGPU_HA_FULL_TUV=1" "MPGPU_HA_FULL_TUV=0" "MPGPU_HA_MIRROR=0" "MPGPU_HA_FPIPE_BLOCKS=0"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st.bin timeout -k 10 200 python3 tools/ha_plan_time.py > $O/st.log 2>&1 &&
python3 tools/ha_stamps_wide.py $O/st.bin > $O/wide.txt && cat $O/wide.txt &&
python3 tools/ha_stamps_blocks.py $O/st.bin 12 > $O/st.txt && rm -f $O/st.bin
