# Round 6: RT tiles interleaved over the XCD ranges (VDS_BATCH_RT_SPREAD) --
# batch / non-codeword GPU tests, then ABBA of the live legs against
# ab/nortspread.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6v
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6v/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6v/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r6c.sh nortspread
