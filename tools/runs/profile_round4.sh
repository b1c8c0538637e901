# Round-4 GPU pass: parity suite, default bench (headline + C4 + live), its
# rocprofv3 kernel-trace summary, PMC traffic passes (k=16, k=32), SQ/LDS
# counters of the k=16 restore, live-shape kernel trace, host bench.
# Usage: bash tools/runs/profile_round4.sh TAG [PART]   (outputs under gpurun_out/prof_TAG/)
#   PART a: steps 1-3 (pytest, bench, rocprof bench); b: steps 4-8; default both
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=${1:-r4}; PART=${2:-ab}; D=gpurun_out/prof_$TAG; mkdir -p $D
if [ "$PART" = b ]; then SKIPA=1; fi
P="rocprofv3 --kernel-trace -T -f csv"
{ [ -n "$SKIPA" ] || {
echo "[1/8] pytest"; timeout -k 10 700 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 &&
echo "[2/8] bench"; timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $D/bench_default.log 2>&1 &&
echo "[3/8] rocprof bench"; timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_rocprof.log 2>&1; }; } &&
{ [ "$PART" = a ] || {
echo "[4/8] fetch/write k16"; timeout -k 10 240 $P --pmc FETCH_SIZE -d $D/pmc_fetch -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_fetch.log 2>&1 &&
timeout -k 10 240 $P --pmc WRITE_SIZE -d $D/pmc_write -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_write.log 2>&1 &&
python tools/pmc_traffic.py $D/pmc_fetch $D/pmc_write 64 $D/traffic.json > /dev/null &&
echo "[5/8] fetch/write k32"; timeout -k 10 240 $P --pmc FETCH_SIZE -d $D/pmc_fetch32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_fetch32.log 2>&1 &&
timeout -k 10 240 $P --pmc WRITE_SIZE -d $D/pmc_write32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_write32.log 2>&1 &&
python tools/pmc_traffic.py $D/pmc_fetch32 $D/pmc_write32 32 $D/traffic_k32.json 32 40 > /dev/null &&
echo "[6/8] sq/lds k16"; timeout -k 10 240 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/pmc_sq -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_sq.log 2>&1 &&
timeout -k 10 240 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/pmc_lds -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_lds.log 2>&1 &&
echo "[7/8] live trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/live -o run -- python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 10 > $D/live_prof.log 2>&1 &&
echo "[7b] live sq"; timeout -k 10 300 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $D/pmc_live_sq -o run -- python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 3 > $D/pmc_live_sq.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $D/pmc_live_sq2 -o run -- python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 3 > $D/pmc_live_sq2.log 2>&1 &&
python tools/pmc_kernels.py $D/pmc_live_kernels.json $D/pmc_live_sq $D/pmc_live_sq2 > $D/pmc_live_kernels.txt &&
echo "[8/8] host"; timeout -k 10 400 python tools/bench_host.py --objects 16 --live 16384 > $D/bench_host.log 2>&1; }; }
rc=$?
echo "rc=$rc"
tail -2 $D/pytest_gpu.log
tail -c 600 $D/bench_default.log
tail -c 600 $D/bench_host.log
exit $rc
