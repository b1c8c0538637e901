# Round 6: host phases with parts of >= 512 (trace) and >= 1024 (trace1k)
# objects, p = 0.02 and 0.25, three alternations.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
for r in 1 2 3; do
  for L in trace trace1k; do
    for p in 0.02 0.25; do
      echo "== $L p=$p round $r" >> gpurun_out/r6y/host_trace.log
      VDS_EC_LIB=ab/$L/libvds_ec.so timeout -k 10 120 python tools/host_trace.py --loss $p >> gpurun_out/r6y/host_trace.log 2>&1 || exit 1
    done
  done
done
grep -E "==|host ms" gpurun_out/r6y/host_trace.log
