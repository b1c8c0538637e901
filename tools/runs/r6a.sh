# Round 6: k = 32 load-issue phase across CUs (s_memrealtime stamps, ab/stamps
# and ab/stamps_st900 = with odd workgroups started 9 us late), then a same-box
# ABBA A/B of the start stagger (VDS_STAGGER / VDS_STAGGER_ENC = 900, 450
# ticks of 10 ns) at k = 32, m = 8, 256 x 64 MiB.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for lib in stamps stamps_st900; do
  for spec in "--k 32 --jit --objects 128" "--k 32 --objects 128"; do
    echo "== $lib $spec"
    VDS_EC_LIB=ab/$lib/libvds_ec.so timeout -k 10 300 python tools/syn_stamps.py $spec > gpurun_out/r6a_stamps.tmp 2>&1 || { cat gpurun_out/r6a_stamps.tmp; exit 1; }
    grep -v amdgpu.ids gpurun_out/r6a_stamps.tmp
  done
done
AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/st900/libvds_ec.so ab/st450/libvds_ec.so > gpurun_out/r6a_ab.log 2>&1 || { cat gpurun_out/r6a_ab.log; exit 1; }
python tools/runs/ab_summary.py gpurun_out/r6a_ab.log
# host planning phases of the live batched calls at p = 0.25 (ab/trace:
# -DVDS_HOST_TRACE=1), then the live legs with per-call spreads (default lib)
VDS_EC_LIB=ab/trace/libvds_ec.so timeout -k 10 300 python tools/host_trace.py --loss 0.25 > gpurun_out/r6a_trace.log 2>&1 || { tail -20 gpurun_out/r6a_trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6a_trace.log | tail -30
timeout -k 10 300 python tools/live_prof.py --loss 0.02 0.25 > gpurun_out/r6a_live.log 2>&1 || { tail -20 gpurun_out/r6a_live.log; exit 1; }
tail -c 3000 gpurun_out/r6a_live.log
