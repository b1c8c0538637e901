# Round 6: RT2 (c) with the extra rows' columns spread over all waves
# (VDS_RT2_SPREAD) -- batch / non-codeword GPU tests, RT stamps, then ABBA of
# the live legs against ab/nospread.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6p
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6p/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6p/pytest.log; [ $rc -eq 0 ] || exit $rc
VDS_EC_LIB=ab/stamps/libvds_ec.so timeout -k 10 200 python tools/rt_stamps.py > gpurun_out/r6p/rt_stamps.txt 2>&1 || exit 1
cat gpurun_out/r6p/rt_stamps.txt
bash tools/runs/r6c.sh nospread
