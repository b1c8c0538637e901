# interpolation phase priorities (VDS_GM2_PRIO variants in build/pN) vs the default (1), k=16, same box
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check --objects 512"
for i in 1 2; do
  $T --tag p1 && for v in 0 3 5 7; do VDS_EC_LIB=build/p$v/libvds_ec.so $T --tag p$v || exit 1; done
done
