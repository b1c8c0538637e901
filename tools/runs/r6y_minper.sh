# Round 6: planner parts of at least 512 objects instead of 1024 (16 parts at
# the live shape's 11,920-object regenerate) -- batch tests, then ABBA of the
# live legs against ab/minper1k.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py > gpurun_out/r6y/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6y/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r6c.sh minper1k
