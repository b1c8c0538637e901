cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/r4b; mkdir -p $D
echo "[1] debug"; timeout -k 10 200 python tools/debug_live_regen.py 16384 0.02 > $D/dbg1.log 2>&1 &&
echo "[2] pytest"; timeout -k 10 700 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 &&
echo "[3] bench"; timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $D/bench_default.log 2>&1 &&
echo "[4] host"; timeout -k 10 400 python tools/bench_host.py --objects 16 --live 16384 > $D/bench_host.log 2>&1
rc=$?; echo rc=$rc; cat $D/dbg1.log; tail -3 $D/pytest_gpu.log; tail -c 5000 $D/bench_default.log; tail -c 1500 $D/bench_host.log; exit $rc
