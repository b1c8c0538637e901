# same-box A/B: two-level interpolation (default build) vs one level (build/gm1, -DVDS_GM2=0),
# with and without the survivor-set kernels; k=16 512 objects and k=32 256 objects
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/gm2
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jit_gpu.py tests/test_parity_gpu.py tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_regenerate_gpu.py > gpurun_out/gm2/pytest.log 2>&1 || { tail -30 gpurun_out/gm2/pytest.log; exit 1; }
tail -2 gpurun_out/gm2/pytest.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  VDS_EC_LIB=build/gm1/libvds_ec.so VDS_EC_JIT=0 $T --objects 512 --tag gm1syn &&
  VDS_EC_JIT=0 $T --objects 512 --tag gm2syn &&
  VDS_EC_LIB=build/gm1/libvds_ec.so $T --objects 512 --tag gm1jit &&
  $T --objects 512 --tag gm2jit || exit 1
done
for i in 1 2; do
  VDS_EC_LIB=build/gm1/libvds_ec.so VDS_EC_JIT=0 $T --k 32 --objects 256 --tag gm1syn32 &&
  VDS_EC_JIT=0 $T --k 32 --objects 256 --tag gm2syn32 &&
  VDS_EC_LIB=build/gm1/libvds_ec.so $T --k 32 --objects 256 --tag gm1jit32 &&
  $T --k 32 --objects 256 --tag gm2jit32 || exit 1
done
