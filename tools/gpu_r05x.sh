# the 6-wave middle shape's range: MPGPU_HA_MID_BLOCKS x MPGPU_HA_TAIL_BLOCKS
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
export TMPDIR=/tmp
for env in "MPGPU_HA_MID_BLOCKS=512" "MPGPU_HA_MID_BLOCKS=512 MPGPU_HA_TAIL_BLOCKS=256" "MPGPU_HA_MID_BLOCKS=384" "MPGPU_HA_MID_BLOCKS=640" "MPGPU_HA_MID_BLOCKS=512 MPGPU_HA_TAIL_BLOCKS=384" "MPGPU_HA_MID_BLOCKS=0" "MPGPU_HA_MID_BLOCKS=512" "MPGPU_HA_MID_BLOCKS=512 MPGPU_HA_TAIL_BLOCKS=256"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
