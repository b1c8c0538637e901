cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/stamps; mkdir -p $D
VDS_EC_LIB=ab/stamps.so timeout -k 10 200 python tools/syn_stamps.py --k 32 --objects 64 > $D/k32.txt 2>&1 &&
VDS_EC_LIB=ab/stamps.so timeout -k 10 200 python tools/syn_stamps.py --k 16 --objects 128 > $D/k16.txt 2>&1
rc=$?; cat $D/k32.txt $D/k16.txt; exit $rc
