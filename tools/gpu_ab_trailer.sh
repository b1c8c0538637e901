cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/ab_trailer; mkdir -p $D
for i in 1 2 3; do
  timeout -k 10 120 python tools/ab_live_encode.py >> $D/ab.log 2>&1 &&
  VDS_EC_ENC_TRAILER=0 timeout -k 10 120 python tools/ab_live_encode.py >> $D/ab.log 2>&1 || exit 1
done
grep tag $D/ab.log
