cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/ht; mkdir -p $D
echo "[1] pytest"; timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_noncodeword_gpu.py tests/test_batch_gpu.py > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
bash tools/runs/gpu_ht.sh
