# Round 6: the k = 16 load study (as r6k_loads.sh at k = 32): stamps of the
# survivor-set and AOT kernels with normal loads, L2-hit reloads and no loads.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6q
for v in stamps stampsL1 stampsL2; do
  for j in "" "--jit"; do
    echo "== $v k16 $j" >> gpurun_out/r6q/stamps.txt
    VDS_EC_LIB=ab/$v/libvds_ec.so timeout -k 10 120 python tools/syn_stamps.py --k 16 --objects 256 $j >> gpurun_out/r6q/stamps.txt 2>&1 || exit 1
  done
done
