cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/r4a; mkdir -p $D
echo "[1] pytest"; timeout -k 10 700 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 &&
echo "[2] bench"; timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $D/bench_default.log 2>&1
rc=$?; echo rc=$rc; tail -3 $D/pytest_gpu.log; tail -c 2500 $D/bench_default.log; exit $rc
