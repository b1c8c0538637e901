set -e
mkdir -p gpurun_out/ls
for v in stamps stampsL1 stampsL2; do
  for j in "" "--jit"; do
    echo "== $v k32 $j" >> gpurun_out/ls/stamps.txt
    VDS_EC_LIB=ab/$v/libvds_ec.so timeout -k 10 120 python tools/syn_stamps.py --k 32 --objects 128 $j >> gpurun_out/ls/stamps.txt 2>&1
  done
done
