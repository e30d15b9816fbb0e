set -u
OUT=gpurun_out/ab4; mkdir -p $OUT
for round in 1 2; do
  for nc in 1 2; do
    AON_F16X3_NCOL=$nc AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_base.so timeout -k 10 120 python tools/prof_mlp.py --precision f16x3 --reps 4 > $OUT/nc$nc.$round.log 2>&1 || exit $?
    echo "ncol $nc round $round: $(grep f16x3 $OUT/nc$nc.$round.log | tail -1)"
  done
done
