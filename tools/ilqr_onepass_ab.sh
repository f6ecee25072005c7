# A/B of mp_ilqr_solve builds (tools/build_variant.sh SUFFIX FLAGS): bash tools/ilqr_onepass_ab.sh _suffix ...
for v in "" "$@" ""; do
  export MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so
  echo "variant [$v]"; timeout -k 10 100 python tools/ilqr_time.py --solve-only 2>&1 | grep solve || exit 1
  timeout -k 10 100 python tools/ilqr_time.py --solve-only 2>&1 | grep solve || exit 1
done
