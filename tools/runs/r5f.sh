# Round 5: two A/Bs on one box, interleaved (run tools/runs/r5_check.sh first): the encode pair plan (ab/nols: LPT only) at k = 16
# (512 objects) and k = 32 (256); the k = 32 restore's LDS-DMA prefetch
# (ab/nodma: VDS_K32_DMA=0) at 256 objects.
cd $GRAFT_REPO_ROOT
row() { python - "$@" <<'PY'
import json, sys
out = [sys.argv[1]]
for f in sys.argv[2:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    out.append(f"{d['config']['k']}: enc {d['encode_ms']} rep {d['repair_ms']} aot {d.get('restore_aot_ms')}")
print(" | ".join(out))
PY
}
for r in 1 2 3; do
  for v in default nols nodma; do
    L=""; [ $v != default ] && L=ab/$v/libvds_ec.so
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --objects 512 --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/ab16_${v}_$r.log 2>&1 || exit $?
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --k 32 --m 8 --objects 256 --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/ab32_${v}_$r.log 2>&1 || exit $?
    row $v gpurun_out/ab16_${v}_$r.log gpurun_out/ab32_${v}_$r.log
  done
done
