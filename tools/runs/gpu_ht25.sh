cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/ht25; mkdir -p $D
VDS_EC_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py --loss 0.25 > $D/ht25.log 2>&1; rc=$?
grep "host ms" $D/ht25.log; grep "restore_batch" $D/ht25.log | tail -2; grep "regenerate_batch" $D/ht25.log | tail -2; exit $rc
