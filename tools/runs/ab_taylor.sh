# k = 32 encode: Taylor step over 8 waves (2 planes each, build/tw) vs 4 waves
# (default); diagnostics d1 (no Taylor step) / d2 (no evaluation) bound what
# those phases cost.  n = 40 and the live n = 64, same box.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T="timeout -k 10 120 python tools/time_kernels.py --align 256"
for i in 1 2; do
  $T --k 32 --objects 256 --tag base --check &&
  VDS_EC_LIB=build/tw $T --k 32 --objects 256 --tag tw --check &&
  VDS_EC_LIB=build/d1 $T --k 32 --objects 256 --tag d1_notaylor &&
  VDS_EC_LIB=build/d2 $T --k 32 --objects 256 --tag d2_noeval &&
  $T --k 32 --n 64 --objects 128 --tag base64 --check &&
  VDS_EC_LIB=build/tw $T --k 32 --n 64 --objects 128 --tag tw64 --check || exit 1
done
