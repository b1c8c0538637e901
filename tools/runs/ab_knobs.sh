# same-box A/B of JIT fill-program knobs (k=16, 512 x 64 MiB), then the default bench line
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/knobs
for i in 1 2; do
  timeout -k 10 120 python tools/time_kernels.py --objects 512 --align 256 --check --tag pb2 || exit 1
  VDS_EC_JIT_PB=3 timeout -k 10 120 python tools/time_kernels.py --objects 512 --align 256 --check --tag pb3 || exit 1
  VDS_EC_JIT_PB=4 VDS_EC_JIT_NOPF=1 timeout -k 10 120 python tools/time_kernels.py --objects 512 --align 256 --check --tag pb4nopf || exit 1
done
timeout -k 10 400 python bench.py > gpurun_out/knobs/bench_default.log 2>&1 || { tail -20 gpurun_out/knobs/bench_default.log; exit 1; }
tail -1 gpurun_out/knobs/bench_default.log
