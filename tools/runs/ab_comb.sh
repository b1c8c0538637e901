# pairs' combination P0(y) + r P1(y) as one Paar Horner step (build/comb1) vs a
# multiply and an XOR (default), same box; encode parity tests first
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/comb
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "encode or golden or full or stream or bench_layout" > gpurun_out/comb/pytest.log 2>&1 || { tail -30 gpurun_out/comb/pytest.log; exit 1; }
VDS_EC_LIB=build/comb1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "encode or golden or full or stream or bench_layout" > gpurun_out/comb/pytest1.log 2>&1 || { tail -30 gpurun_out/comb/pytest1.log; exit 1; }
tail -1 gpurun_out/comb/pytest.log; tail -1 gpurun_out/comb/pytest1.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2 3; do
  $T --objects 512 --tag comb0_16 &&
  VDS_EC_LIB=build/comb1 $T --objects 512 --tag comb1_16 &&
  $T --k 32 --objects 256 --tag comb0_40 &&
  VDS_EC_LIB=build/comb1 $T --k 32 --objects 256 --tag comb1_40 || exit 1
done
