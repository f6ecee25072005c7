#!/bin/bash
# Build an A/B variant of libmpgpu with extra compile flags into motionplanning_amd/lib/libmpgpu_SUFFIX.so
# (tools/mppi_ab.sh then selects it with MPGPU_LIB).
# usage: bash tools/build_variant.sh SUFFIX "-DFOO -DBAR"
set -e
SUF=$1
EXTRA=$2
cd "$(dirname "$0")/../motionplanning_amd/csrc"
B=build_$SUF
mkdir -p $B
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I../../include -Wno-unused-result -Wno-unused-value"
pids=()
for f in *.hip; do
  n=${f%.hip}
  extra_file=""
  [ "$n" = "ilqr" ] && extra_file="-mllvm -amdgpu-sched-strategy=iterative-ilp"
  $HIPCC $FLAGS $extra_file $EXTRA -c $f -o $B/$n.o &
  pids+=($!)
done
$HIPCC $FLAGS $EXTRA -x hip -c runtime.cpp -o $B/runtime.o &
pids+=($!)
$HIPCC $FLAGS $EXTRA -x hip -c comm.cpp -o $B/comm.o &
pids+=($!)
for p in "${pids[@]}"; do wait $p; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -pthread -o ../lib/libmpgpu_$SUF.so $B/*.o -ldl
rm -rf $B
echo "built motionplanning_amd/lib/libmpgpu_$SUF.so"
