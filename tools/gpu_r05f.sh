set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -3 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && cat $O/lone.log &&
MPGPU_HA_TAIL_RSH=0 timeout -k 10 200 python3 tools/ha_lone.py > $O/lone_norsh.log 2>&1 && cat $O/lone_norsh.log &&
timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && cat $O/ha.log &&
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st.log 2>&1 &&
python3 tools/ha_stamps_blocks.py $O/st.bin 4 > $O/st.txt || exit 1
for v in "" _coh _ocml ""; do
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 bench.py --steps 100 --warmup 200 --no-cpu --no-extras --no-single > $O/bench$v.json 2> $O/bench$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/bench$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'])"
done
for v in "" _pipe3 _pipe4; do
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ilqr_time.py --solve-only > $O/ilqr$v.log 2>&1 || exit 1
  echo "== ilqr$v"; tail -3 $O/ilqr$v.log
done
