# Full GPU round: parity suite, PMC traffic passes, the default bench line and
# its rocprofv3 kernel-trace summary, plus the C4 (k=32) and C5 (host-memory)
# lines.  Usage: bash tools/runs/profile_round.sh TAG
# Outputs under gpurun_out/prof_TAG/ (copy the summaries into profiles/).
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=${1:-r1}; D=gpurun_out/prof_$TAG; mkdir -p $D
P="rocprofv3 --kernel-trace -T -f csv"
echo "[1/9] pytest"; timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 &&
echo "[2/9] fetch"; timeout -k 10 240 $P --pmc FETCH_SIZE -d $D/pmc_fetch -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_fetch.log 2>&1 &&
echo "[3/9] write"; timeout -k 10 240 $P --pmc WRITE_SIZE -d $D/pmc_write -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_write.log 2>&1 &&
echo "[4/9] sq"; timeout -k 10 240 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/pmc_sq -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_sq.log 2>&1 &&
echo "[5/9] lds"; timeout -k 10 240 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/pmc_lds -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > $D/pmc_lds.log 2>&1 &&
python tools/pmc_traffic.py $D/pmc_fetch $D/pmc_write 64 $D/traffic.json > /dev/null &&
echo "[6/9] bench"; timeout -k 10 400 python bench.py --traffic-json $D/traffic.json > $D/bench_default.log 2>&1 &&
echo "[7/9] rocprof bench"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python bench.py --traffic-json $D/traffic.json --no-cpu-baseline > $D/bench_rocprof.log 2>&1 &&
echo "[8/9] k32"; timeout -k 10 240 $P --pmc FETCH_SIZE -d $D/pmc_fetch32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_fetch32.log 2>&1 &&
timeout -k 10 240 $P --pmc WRITE_SIZE -d $D/pmc_write32 -o run -- python tools/prof_kernels.py --k 32 --m 8 --objects 32 --iters 2 > $D/pmc_write32.log 2>&1 &&
python tools/pmc_traffic.py $D/pmc_fetch32 $D/pmc_write32 32 $D/traffic_k32.json 32 40 > /dev/null &&
timeout -k 10 400 python bench.py --k 32 --m 8 --objects 512 --no-cpu-baseline --traffic-json $D/traffic_k32.json > $D/bench_k32.log 2>&1 &&
echo "[9/9] host"; timeout -k 10 400 python tools/bench_host.py --objects 16 --live 16384 > $D/bench_host.log 2>&1 &&
echo "[+] pcie duplex / drop-in loop"; timeout -k 10 120 tools/ubench/pcie_duplex 256 > $D/pcie_duplex.json 2>&1 &&
timeout -k 10 120 tools/dropin_loop 200 > $D/dropin_loop.json 2>&1
rc=$?
echo "rc=$rc"
tail -2 $D/pytest_gpu.log
tail -1 $D/bench_default.log
tail -1 $D/bench_k32.log
tail -1 $D/bench_host.log
cat $D/pcie_duplex.json $D/dropin_loop.json
exit $rc
