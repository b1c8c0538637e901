# Round 6: the k = 32 N-point syndrome class of the batched restore routed
# to the RT batch (ab/n2rt: -DVDS_BATCH_N_TO_RT=1) -- batch / non-codeword GPU
# tests with that library, then ABBA of the live legs against the default.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
VDS_EC_LIB=ab/n2rt/libvds_ec.so timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6j_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6j_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r6c.sh n2rt
