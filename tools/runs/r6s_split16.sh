# Round 6: k = 16 survivor-set kernel with half of the next tile's loads issued
# before the fill (VDS_K16_SPLITPF) -- parity of the survivor-set kernels, then
# ABBA at 512 x 64 MiB against ab/nosplit.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6s
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_noncodeword_gpu.py tests/test_jit_gpu.py > gpurun_out/r6s/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6s/pytest.log; [ $rc -eq 0 ] || exit $rc
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/nosplit/libvds_ec.so > gpurun_out/r6s/ab.log 2>&1
cat gpurun_out/r6s/ab.log; python tools/runs/ab_summary.py gpurun_out/r6s/ab.log
