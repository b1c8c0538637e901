# Round 5: k = 16 survivor-set kernels store only the survivors the
# interpolation reads (points < k; none when regenerating) -- default --
# against ab/prev (HEAD before); GPU suite first; ABBA, restore and the
# bench's regenerate leg.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5n; mkdir -p $D
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
cat $D/ab_k16.log; python tools/runs/ab_summary.py $D/ab_k16.log
grep -h '"regenerate_GiBps"' gpurun_out/abk_*_[123][ab].log | python -c "
import json,sys
for l in sys.stdin: pass
" ; for f in gpurun_out/abk_*_[123][ab].log; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], 'regen', d.get('regenerate_ms'))"; done
