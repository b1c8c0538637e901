cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/hth; mkdir -p $D
for t in 8 12 16 8; do for p in 0.02 0.25; do
  VDS_EC_HOST_THREADS=$t VDS_EC_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py --loss $p > $D/ht_${t}_$p.log 2>&1 || exit 1
  echo "== threads $t loss $p"; grep "host ms" $D/ht_${t}_$p.log; grep "regenerate_batch" $D/ht_${t}_$p.log | tail -1
done; done
