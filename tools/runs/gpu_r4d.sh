cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/r4d; mkdir -p $D
echo "[1] pytest batch"; timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_host_pinned_gpu.py tests/test_parity_gpu.py > $D/pytest_gpu.log 2>&1 &&
echo "[2] live prof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/live -o run -- python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 10 > $D/live_prof.log 2>&1 &&
echo "[3] host"; timeout -k 10 400 python tools/bench_host.py --objects 16 --live 16384 > $D/bench_host.log 2>&1 &&
echo "[4] host dma"; VDS_EC_PIN_D2H=dma timeout -k 10 400 python tools/bench_host.py --objects 16 --live 16384 > $D/bench_host_dma.log 2>&1
rc=$?; echo rc=$rc; tail -2 $D/pytest_gpu.log; tail -c 1200 $D/live_prof.log; tail -c 700 $D/bench_host.log; tail -c 700 $D/bench_host_dma.log; exit $rc
