# Round 6: dual syndrome tiles for the regenerate too -- batch / non-codeword
# GPU tests, RT-kernel stamps (tools/rt_stamps.py), then ABBA of the live legs
# against ab/nodual.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6o
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6o/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6o/pytest.log; [ $rc -eq 0 ] || exit $rc
VDS_EC_LIB=ab/stamps/libvds_ec.so timeout -k 10 200 python tools/rt_stamps.py > gpurun_out/r6o/rt_stamps.txt 2>&1 || exit 1
cat gpurun_out/r6o/rt_stamps.txt
bash tools/runs/r6c.sh nodual
