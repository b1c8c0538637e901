# Round 5 checkpoint: the GPU suite, then the default bench line (headline,
# C4, live shape, CPU baseline) and the per-call latency tool.
#   bash tools/runs/r5_check.sh TAG      (outputs under gpurun_out/TAG/)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
D=gpurun_out/${1:-r5chk}; mkdir -p $D
echo "[1/3] pytest"; timeout -k 10 800 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1
rc=$?; tail -2 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "[2/3] bench"; timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $D/bench_default.log 2>&1 || exit $?
tail -c 400 $D/bench_default.log
echo "[3/3] latency"; timeout -k 10 120 tools/dropin_loop 400 > $D/dropin_loop.json 2>&1 || exit $?
cat $D/dropin_loop.json
