# Round-6 closing GPU pass (run at the final commit), in two parts that each
# fit one gpurun call:
#   bash tools/runs/profile_round6.sh TAG a   pytest, default bench (+CPU baseline),
#                                             rocprofv3 --kernel-trace --stats of the
#                                             bench (no align16 leg, so every kernel
#                                             symbol has one launch size), the
#                                             rocprof-vs-HIP-event table
#   bash tools/runs/profile_round6.sh TAG b   PMC traffic (k=16, k=32), SQ / LDS
#                                             counters, live-shape trace and SQ,
#                                             host (PCIe) rates, per-call latency
# Outputs under gpurun_out/prof_TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=${1:-r6}; PART=${2:-a}; D=gpurun_out/prof_$TAG; mkdir -p $D
P="rocprofv3 --kernel-trace -T -f csv"
if [ "$PART" = a ]; then
  echo "[a1] pytest"; timeout -k 10 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 &&
  echo "[a2] bench"; timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $D/bench_default.log 2>&1 &&
  echo "[a3] rocprof bench"; timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-align16 > $D/bench_rocprof.log 2>&1 &&
  python tools/rocprof_vs_bench.py $D/bench_rocprof.log $(find $D/trace -name 'run_kernel_stats.csv' | head -1) > $D/roofline_vs_rocprof.txt
  rc=$?
  tail -2 $D/pytest_gpu.log; tail -c 300 $D/bench_default.log; cat $D/roofline_vs_rocprof.txt
  exit $rc
fi
echo "[b1] fetch/write k16"; timeout -k 10 240 $P --pmc FETCH_SIZE -d $D/pmc_fetch -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_fetch.log 2>&1 &&
timeout -k 10 240 $P --pmc WRITE_SIZE -d $D/pmc_write -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_write.log 2>&1 &&
python tools/pmc_traffic.py $(find $D/pmc_fetch -name '*counter_collection.csv' -printf '%h\n' | head -1) $(find $D/pmc_write -name '*counter_collection.csv' -printf '%h\n' | head -1) 64 $D/traffic.json > /dev/null &&
echo "[b2] fetch/write k32"; timeout -k 10 240 $P --pmc FETCH_SIZE -d $D/pmc_fetch32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_fetch32.log 2>&1 &&
timeout -k 10 240 $P --pmc WRITE_SIZE -d $D/pmc_write32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_write32.log 2>&1 &&
python tools/pmc_traffic.py $(find $D/pmc_fetch32 -name '*counter_collection.csv' -printf '%h\n' | head -1) $(find $D/pmc_write32 -name '*counter_collection.csv' -printf '%h\n' | head -1) 32 $D/traffic_k32.json 32 40 > /dev/null &&
echo "[b3] sq/lds k16"; timeout -k 10 240 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/pmc_sq -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_sq.log 2>&1 &&
timeout -k 10 240 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/pmc_lds -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_lds.log 2>&1 &&
echo "[b4] sq/lds k32"; timeout -k 10 240 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/pmc_sq32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_sq32.log 2>&1 &&
timeout -k 10 240 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/pmc_lds32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_lds32.log 2>&1 &&
echo "[b5] live trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/live -o run -- python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 10 > $D/live_prof.log 2>&1 &&
echo "[b5b] live sq/lds (RT + MULTI at p = 0.25)"; timeout -k 10 240 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/pmc_live_sq -o run -- python tools/live_prof.py --objects 16384 --loss 0.25 --steps 2 > $D/pmc_live_sq.log 2>&1 &&
timeout -k 10 240 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/pmc_live_lds -o run -- python tools/live_prof.py --objects 16384 --loss 0.25 --steps 2 > $D/pmc_live_lds.log 2>&1 &&
echo "[b6] host + latency"; timeout -k 10 400 python tools/bench_host.py --objects 16 --live 16384 > $D/bench_host.log 2>&1 &&
timeout -k 10 120 tools/dropin_loop 400 > $D/dropin_loop.json 2>&1
rc=$?
echo "rc=$rc"
tail -c 600 $D/bench_host.log
cat $D/dropin_loop.json
exit $rc
