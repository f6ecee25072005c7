# shape thresholds with the persistent tail: MPGPU_HA_TAIL_BLOCKS (full width -> 12-wave tail) and the middle shape
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp
for env in "MPGPU_HA_TAIL_BLOCKS=512" "MPGPU_HA_TAIL_BLOCKS=768" "MPGPU_HA_TAIL_BLOCKS=1024" "MPGPU_HA_TAIL_BLOCKS=1536" "MPGPU_HA_TAIL_BLOCKS=2048" "MPGPU_HA_MID_BLOCKS=1024" "MPGPU_HA_MID_BLOCKS=2048" "MPGPU_HA_TAIL_BLOCKS=512"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && tail -5 $O/ha.log || exit 1
done
