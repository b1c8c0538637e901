cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/rt2b; mkdir -p $D
for r in 8 4 1; do for v in 1 0; do
  VDS_EC_RT2=$v timeout -k 10 120 python tools/rt2_bench.py --rows $r >> $D/rt2b.log 2>&1 || { tail -5 $D/rt2b.log; exit 1; }
done; done
cat $D/rt2b.log | grep rt2
