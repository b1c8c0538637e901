# encode at fewer workgroups per CU (VDS_EC_ENC_LDS_EXTRA pads the LDS): is the
# k = 32 encode (1 workgroup per CU) limited by phase serialisation?
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/occ
T="timeout -k 10 120 python tools/time_kernels.py --align 256"
for i in 1 2; do
  $T --objects 512 --tag k16_2wg &&
  VDS_EC_ENC_LDS_EXTRA=20000 $T --objects 512 --tag k16_1wg &&
  $T --k 32 --objects 256 --tag k32 || exit 1
done
