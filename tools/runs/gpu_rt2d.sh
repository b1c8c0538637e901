cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/rt2d; mkdir -p $D
echo "[1] pytest"; timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_noncodeword_gpu.py tests/test_batch_gpu.py > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
for r in 8 4; do for v in 1 0; do VDS_EC_RT2=$v timeout -k 10 120 python tools/rt2_bench.py --rows $r >> $D/rt2b.log 2>&1 || { tail -5 $D/rt2b.log; exit 1; }; done; done
grep rt2 $D/rt2b.log
