# k = 32 stage C after the interpolation branches with the next tile's loads
# issued between its reads (VDS_K32_EARLYC): parity, stamps, then ABBA timing
# against the previous form (ab/earlyc0).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6l
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_noncodeword_gpu.py -m gpu > gpurun_out/r6l/pytest.log 2>&1
tail -2 gpurun_out/r6l/pytest.log
for v in stamps stampsE; do
  for j in "" "--jit"; do
    echo "== $v k32 $j" >> gpurun_out/r6l/stamps.txt
    VDS_EC_LIB=ab/$v/libvds_ec.so timeout -k 10 120 python tools/syn_stamps.py --k 32 --objects 128 $j >> gpurun_out/r6l/stamps.txt 2>&1
  done
done
AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/earlyc0/libvds_ec.so > gpurun_out/r6l/ab.log 2>&1
cat gpurun_out/r6l/ab.log
