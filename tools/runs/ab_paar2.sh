# with the Paar Horner steps: one- vs two-level split at n = 40 and n = 64
# (VDS_EC_ENCODE_PATH), same box; encode parity tests of both paths first
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/paar2
P="timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k"
$P "encode or golden or full or stream or bench_layout" > gpurun_out/paar2/pytest.log 2>&1 || { tail -30 gpurun_out/paar2/pytest.log; exit 1; }
VDS_EC_ENCODE_PATH=q $P "encode or golden or full or stream or bench_layout" > gpurun_out/paar2/pytest_q.log 2>&1 || { tail -30 gpurun_out/paar2/pytest_q.log; exit 1; }
tail -1 gpurun_out/paar2/pytest.log; tail -1 gpurun_out/paar2/pytest_q.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  $T --k 32 --objects 256 --tag pair40 &&
  VDS_EC_ENCODE_PATH=q $T --k 32 --objects 256 --tag quad40 &&
  $T --k 32 --n 64 --objects 128 --tag quad64 &&
  VDS_EC_ENCODE_PATH=pair $T --k 32 --n 64 --objects 128 --tag pair64 &&
  $T --objects 512 --tag pair16 &&
  VDS_EC_ENCODE_PATH=q $T --objects 512 --tag quad16 || exit 1
done
