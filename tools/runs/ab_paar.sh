# encode Horner steps as Paar XOR programs (default build) vs the row form
# (build/rows, -DVDS_ENC_PAAR=0), same box; encode parity tests first
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/paar
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "encode or golden or full or stream or bench_layout" > gpurun_out/paar/pytest.log 2>&1 || { tail -30 gpurun_out/paar/pytest.log; exit 1; }
tail -1 gpurun_out/paar/pytest.log
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  VDS_EC_LIB=build/rows $T --k 32 --objects 256 --tag rows40 &&
  $T --k 32 --objects 256 --tag paar40 &&
  VDS_EC_LIB=build/rows $T --k 32 --n 64 --objects 128 --tag rows64 &&
  $T --k 32 --n 64 --objects 128 --tag paar64 &&
  VDS_EC_LIB=build/rows $T --objects 512 --tag rows16 &&
  $T --objects 512 --tag paar16 || exit 1
done
for i in 1 2; do
  VDS_EC_LIB=build/rows timeout -k 10 300 python bench.py --steps 5 --objects 64 --no-cpu-baseline --no-align16 > gpurun_out/paar/live_rows$i.log 2>&1 &&
  timeout -k 10 300 python bench.py --steps 5 --objects 64 --no-cpu-baseline --no-align16 > gpurun_out/paar/live_paar$i.log 2>&1 || exit 1
  for v in rows paar; do python -c "import json;d=json.loads(open('gpurun_out/paar/live_${v}$i.log').read().splitlines()[-1])['live_shape'];print('$v live', d['encode_GiBps'], d['sha256_object_GiBps'])"; done
done
