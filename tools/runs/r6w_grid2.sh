# Round 6: batch kernels launched with twice the resident workgroups
# (-DVDS_BATCH_GRID_X=2: the dispatcher hands later workgroups to the CUs
# that finish first) -- batch tests with that library, then ABBA of the live
# legs (r6c.sh's "default" is the shipped build).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6w
VDS_EC_LIB=ab/grid2/libvds_ec.so timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py > gpurun_out/r6w/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6w/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r6c.sh grid2
