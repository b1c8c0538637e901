# LDS bank-conflict fixes (swizzled XOR atomics + ds_read_b64 copy-out) vs build/swz0 (neither), same box
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/swz
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jit_gpu.py tests/test_parity_gpu.py -k "jit or syndrome or restore or full" > gpurun_out/swz/pytest.log 2>&1 || { tail -30 gpurun_out/swz/pytest.log; exit 1; }
tail -1 gpurun_out/swz/pytest.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2 3; do
  VDS_EC_LIB=build/swz0/libvds_ec.so $T --objects 512 --tag old16 && $T --objects 512 --tag swz16 || exit 1
done
for i in 1 2; do
  VDS_EC_LIB=build/swz0/libvds_ec.so $T --k 32 --objects 256 --tag old32 && $T --k 32 --objects 256 --tag swz32 || exit 1
done
P="timeout -s KILL 60 rocprofv3 --kernel-trace -T -f csv"
$P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d gpurun_out/swz/pmc -o run -- python tools/prof_kernels.py --objects 64 --iters 2 --only restore > gpurun_out/swz/pmc.log 2>&1 || exit 1
python tools/pmc_summary.py vds_ec_jit gpurun_out/swz/pmc
