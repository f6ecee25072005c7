# which run segfaults at exit under rocprofv3 --pmc: the Hybrid A* plan without / with the cooperative persistent tail
set -o pipefail
O=gpurun_out/r05z2; mkdir -p $O
export TMPDIR=/tmp
MPGPU_HA_PERSIST=0 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES -d $O/p0 -o run --output-format csv -- python3 tools/ha_lone.py 1 > $O/p0.log 2>&1; echo "persist=0 exit $?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t1 -o run --output-format csv -- python3 tools/ha_lone.py 1 > $O/t1.log 2>&1; echo "persist=1 kernel-trace exit $?"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 tools/ha_lone.py 1 > $O/p1.log 2>&1; echo "persist=1 pmc exit $?"
