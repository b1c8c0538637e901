# survivor-set kernels: GPU tests, then fill forms (3 interleaved rounds: row, scatter spb1, scatter spb2)
# and regenerate on the syndrome kernel vs its run-time compiled twin
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/scat2
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jit_gpu.py tests/test_noncodeword_gpu.py tests/test_regenerate_gpu.py > gpurun_out/scat2/pytest.log 2>&1 || { tail -30 gpurun_out/scat2/pytest.log; exit 1; }
tail -1 gpurun_out/scat2/pytest.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2 3; do
  VDS_EC_JIT_SCATTER=0 $T --objects 512 --tag row16 && VDS_EC_JIT_SPB=1 $T --objects 512 --tag scat1_16 &&
  VDS_EC_JIT_SPB=2 $T --objects 512 --tag scat2_16 || exit 1
done
for i in 1 2; do
  VDS_EC_JIT_SCATTER=0 $T --k 32 --objects 256 --tag row32 && VDS_EC_JIT_SPB=1 $T --k 32 --objects 256 --tag scat1_32 &&
  VDS_EC_JIT_SPB=2 $T --k 32 --objects 256 --tag scat2_32 || exit 1
done
B="timeout -k 10 300 python bench.py --objects 256 --no-live --no-cpu-baseline --no-align16"
VDS_EC_JIT=0 $B > gpurun_out/scat2/b_syn.log 2>&1 && $B > gpurun_out/scat2/b_jit.log 2>&1 || exit 1
for v in syn jit; do python -c "import json;d=json.loads(open('gpurun_out/scat2/b_$v.log').read().splitlines()[-1]);print('regen $v', d['regenerate_GiBps'], d['regenerate_ms'], d['repair_ms'], d['restore_kernel'])"; done
