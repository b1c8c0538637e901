cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/ht; mkdir -p $D
for p in 0.02 0.25; do VDS_EC_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py --loss $p > $D/ht_$p.log 2>&1 || exit 1
echo "== $p"; grep "host ms" $D/ht_$p.log; grep "restore_batch" $D/ht_$p.log | tail -2; grep "regenerate_batch" $D/ht_$p.log | tail -2; done
