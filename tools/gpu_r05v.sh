# shape thresholds once the host sees the live count promptly (the mirror): MPGPU_HA_TAIL_BLOCKS x FPIPE x MIRROR
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
for env in "MPGPU_HA_MIRROR=0" "MPGPU_HA_FPIPE_BLOCKS=0" "MPGPU_HA_FPIPE_BLOCKS=0 MPGPU_HA_TAIL_BLOCKS=256" "MPGPU_HA_FPIPE_BLOCKS=0 MPGPU_HA_TAIL_BLOCKS=384" "MPGPU_HA_TAIL_BLOCKS=256" "MPGPU_HA_MIRROR=0 MPGPU_HA_FPIPE_BLOCKS=0" "MPGPU_HA_MIRROR=0 MPGPU_HA_TAIL_BLOCKS=256" "MPGPU_HA_MIRROR=0"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -3 || exit 1
done
