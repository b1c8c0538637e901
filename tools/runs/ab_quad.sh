# encode: two-level (quad) vs one-level (pair) split, same box; parity tests of the encode paths first
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/quad
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "encode or golden or full or stream or bench_layout" > gpurun_out/quad/pytest.log 2>&1 || { tail -30 gpurun_out/quad/pytest.log; exit 1; }
VDS_EC_ENCODE_PATH=q timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "encode or golden or full or stream or bench_layout" > gpurun_out/quad/pytest_q16.log 2>&1 || { tail -30 gpurun_out/quad/pytest_q16.log; exit 1; }
tail -1 gpurun_out/quad/pytest.log; tail -1 gpurun_out/quad/pytest_q16.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  VDS_EC_ENCODE_PATH=pair $T --k 32 --objects 256 --tag pair32 &&
  $T --k 32 --objects 256 --tag quad32 &&
  $T --objects 512 --tag pair16 &&
  VDS_EC_ENCODE_PATH=q $T --objects 512 --tag quad16 || exit 1
done
for i in 1 2; do
  VDS_EC_ENCODE_PATH=pair timeout -k 10 300 python bench.py --steps 5 --objects 64 --no-cpu-baseline --no-align16 > gpurun_out/quad/live_pair$i.log 2>&1 &&
  timeout -k 10 300 python bench.py --steps 5 --objects 64 --no-cpu-baseline --no-align16 > gpurun_out/quad/live_quad$i.log 2>&1 || exit 1
  for v in pair quad; do python -c "import json;d=json.loads(open('gpurun_out/quad/live_${v}$i.log').read().splitlines()[-1])['live_shape'];print('$v live', d['encode_GiBps'], d['sha256_object_GiBps'])"; done
done
