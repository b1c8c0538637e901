# survivor-set kernel: scatter (column) fill vs row fill, k=16 512 objects / k=32 256 objects, same box
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/scatter
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jit_gpu.py > gpurun_out/scatter/pytest.log 2>&1 || { tail -30 gpurun_out/scatter/pytest.log; exit 1; }
tail -1 gpurun_out/scatter/pytest.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  VDS_EC_JIT_SCATTER=0 $T --objects 512 --tag row16 && $T --objects 512 --tag scat16 &&
  VDS_EC_JIT_SCATTER=0 $T --k 32 --objects 256 --tag row32 && $T --k 32 --objects 256 --tag scat32 || exit 1
done
VDS_EC_JIT_SPB=2 $T --objects 512 --tag scat16spb2 && VDS_EC_JIT_SPB=2 $T --k 32 --objects 256 --tag scat32spb2
