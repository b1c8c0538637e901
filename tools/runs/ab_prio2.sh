# scatter-fill priority (f1), stage-C priority (c9), both (f1c9) vs the default, k=16, same box
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check --objects 512"
for i in 1 2 3; do
  $T --tag base && for v in f1 c9 f1c9; do VDS_EC_LIB=build/$v/libvds_ec.so $T --tag $v || exit 1; done
done
