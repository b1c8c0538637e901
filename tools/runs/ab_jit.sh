# JIT restore: GPU tests, then same-box A/B of the repair (k_restore_syn vs the survivor set's kernel)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/jit
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_jit_gpu.py tests/test_parity_gpu.py -k "jit or syndrome or restore" > gpurun_out/jit/pytest.log 2>&1 || { tail -30 gpurun_out/jit/pytest.log; exit 1; }
tail -3 gpurun_out/jit/pytest.log
for i in 1 2; do
VDS_EC_JIT=0 timeout -k 10 120 python tools/time_kernels.py --objects 512 --align 256 --check --tag syn &&
timeout -k 10 120 python tools/time_kernels.py --objects 512 --align 256 --check --tag jit || exit 1
done
VDS_EC_JIT=0 timeout -k 10 120 python tools/time_kernels.py --k 32 --objects 256 --align 256 --check --tag syn32 &&
timeout -k 10 120 python tools/time_kernels.py --k 32 --objects 256 --align 256 --check --tag jit32
