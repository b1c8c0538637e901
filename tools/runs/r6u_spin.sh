# Round 6: spin-then-sleep planner pool (VDS_POOL_SPIN_US) -- batch tests,
# host phases with and without the spin (trace builds), ABBA of the live legs
# against ab/nospin.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6u
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py > gpurun_out/r6u/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6u/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in trace tracens; do
  for p in 0.02 0.25; do
    echo "== $L p=$p" >> gpurun_out/r6u/host_trace.log
    VDS_EC_LIB=ab/$L/libvds_ec.so timeout -k 10 120 python tools/host_trace.py --loss $p >> gpurun_out/r6u/host_trace.log 2>&1 || exit 1
  done
done
grep -E "==|host ms" gpurun_out/r6u/host_trace.log
bash tools/runs/r6c.sh nospin
