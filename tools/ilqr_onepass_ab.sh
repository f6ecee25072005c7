for v in "" _op512 _op1024 ""; do
  export MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so
  echo "variant [$v]"; timeout -k 10 100 python tools/ilqr_time.py --solve-only 2>&1 | grep solve || exit 1
  timeout -k 10 100 python tools/ilqr_time.py --solve-only 2>&1 | grep solve || exit 1
done
