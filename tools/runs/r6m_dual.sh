# Round 6: dual syndrome tiles (VDS_BATCH_DUAL) -- batch / non-codeword GPU
# tests with the default library, then ABBA of the live legs against
# ab/nodual (-DVDS_BATCH_DUAL=0).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6m/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6m/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r6c.sh nodual
