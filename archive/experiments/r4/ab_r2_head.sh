#!/bin/bash
# Same-box alternating A/B: round-2 tree (abtree/r2 = git 7120714, its own built _C.so) vs HEAD,
# headline + config2, 3 rounds each.  Writes gpurun_out/r4a/.
set -o pipefail
OUT=gpurun_out/r4a; mkdir -p $OUT
cd /root/repo
rocm-smi --showclocks > $OUT/smi_before.txt 2>&1 || true
for i in 1 2 3; do
  ( cd abtree/r2 && timeout -k 10 300 python bench.py --steps 10 --warmup 3 > ../../$OUT/r2_$i.json 2> ../../$OUT/r2_$i.err ) || { echo "r2 run $i failed rc=$?"; exit 1; }
  echo "r2 $i: $(cut -c1-200 $OUT/r2_$i.json)"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2-mb4 off > $OUT/head_$i.json 2> $OUT/head_$i.err || { echo "head run $i failed rc=$?"; exit 1; }
  echo "head $i: $(cut -c1-200 $OUT/head_$i.json)"
done
