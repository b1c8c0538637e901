cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/ab_trailer; mkdir -p $D
for i in 1 2 3; do
  timeout -k 10 120 python tools/ab_live_encode.py >> $D/ab.log 2>&1 &&
  VDS_EC_ENC_TRAILER=0 timeout -k 10 120 python tools/ab_live_encode.py >> $D/ab.log 2>&1 || exit 1
done
grep tag $D/ab.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  $T --objects 512 --tag comb0_16 && VDS_EC_LIB=ab/comb1.so $T --objects 512 --tag comb1_16 &&
  $T --k 32 --objects 256 --tag comb0_40 && VDS_EC_LIB=ab/comb1.so $T --k 32 --objects 256 --tag comb1_40 || exit 1
done
