# Round 6: RT2 rows read once when both halves borrow the same point, objects
# paired by their borrowed points -- batch tests, RT stamps, ABBA of the live
# legs against ab/nosame (-DVDS_RT2_SAME=0 -DVDS_BATCH_RT2_PAIR=0).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6r
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6r/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6r/pytest.log; [ $rc -eq 0 ] || exit $rc
VDS_EC_LIB=ab/stamps/libvds_ec.so timeout -k 10 200 python tools/rt_stamps.py > gpurun_out/r6r/rt_stamps.txt 2>&1 || exit 1
cat gpurun_out/r6r/rt_stamps.txt
bash tools/runs/r6c.sh nosame
