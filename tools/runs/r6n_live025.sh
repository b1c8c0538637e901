# Round 6: live p = 0.25 after the dual tiles -- per-kernel device time
# (rocprofv3 kernel trace) and the host phases of the batched calls
# (ab/trace: -DVDS_HOST_TRACE=1).
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r6n/prof -o live -- python3 tools/live_prof.py --loss 0.25 > gpurun_out/r6n/live_prof.log 2>&1
VDS_EC_LIB=ab/trace/libvds_ec.so timeout -k 10 120 python tools/host_trace.py --loss 0.25 > gpurun_out/r6n/host_trace.log 2>&1
find gpurun_out/r6n/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r6n/live_kernel_stats.csv
