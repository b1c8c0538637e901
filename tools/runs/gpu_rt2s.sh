cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/rt2s; mkdir -p $D
for r in 8 1; do for v in 1 0; do
  echo "== rows $r rt2 $v" >> $D/s.log
  VDS_EC_LIB=ab/stamps.so VDS_EC_RT2=$v timeout -k 10 120 python tools/rt2_bench.py --rows $r --steps 3 >> $D/s.log 2>&1 || { tail -5 $D/s.log; exit 1; }
done; done
grep -v amdgpu.ids $D/s.log
