# Round 5: C4 full-size golden tests, phase stamps of the k = 32 / k = 16
# survivor-set kernels and the k = 32 syndrome kernel (ab/stamps:
# VDS_DIAG_STAMPS=1), then the C4 bench at 256 objects with the default build.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "c4_full or golden" > gpurun_out/r5b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5b_pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "--k 32 --jit --objects 64" "--k 16 --jit --objects 128" "--k 32 --objects 64"; do
  echo "== $spec"
  VDS_EC_LIB=ab/stamps/libvds_ec.so timeout -k 10 300 python tools/syn_stamps.py $spec 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python bench.py --k 32 --m 8 --objects 256 --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/r5b_bench32.log 2>&1 || exit 1
tail -c 1500 gpurun_out/r5b_bench32.log
