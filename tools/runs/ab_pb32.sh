# k=32 survivor-set kernel: fill block size A/B (256 x 64 MiB), same box
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T="timeout -k 10 120 python tools/time_kernels.py --k 32 --objects 256 --align 256 --check"
for i in 1 2; do
  VDS_EC_JIT_PB=2 $T --tag pb2 && VDS_EC_JIT_PB=3 $T --tag pb3 && VDS_EC_JIT_PB=4 VDS_EC_JIT_NOPF=1 $T --tag pb4nopf &&
  VDS_EC_JIT_PB=2 VDS_EC_JIT_NOPF=1 $T --tag pb2nopf || exit 1
done
