# new shape defaults (6-wave middle shape at <= 512 blocks, tail at <= 256): HA GPU tests, then the middle's range
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_MID_BLOCKS=512" "MPGPU_HA_MID_BLOCKS=640" "MPGPU_HA_MID_BLOCKS=768" "MPGPU_HA_MID_BLOCKS=512 MPGPU_HA_TAIL_BLOCKS=512" "MPGPU_HA_MID_BLOCKS=512" "MPGPU_HA_MID_BLOCKS=640" "MPGPU_HA_MID_BLOCKS=768"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && cat $O/lone.log
