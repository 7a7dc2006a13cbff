#!/bin/bash
# Native fp32 MFMA vs bf16x6 (hyres_conv_tuning key 7) on the implicit-GEMM conv families of the fp32 C2 step
# (bs 16): short-K 1x1 layers of the 128-channel ResidualUnits at 128^2 / 64^2, the AttentionBlock(192) units at
# 32^2, a g_a 5x5 stride-2 layer. One line per (shape, mode) from scripts/conv_micro.py.
set -e
for shape in "--H 128 --Ci 128 --Co 64 --K 1 --relu" "--H 128 --Ci 64 --Co 128 --K 1 --res --relu" \
             "--H 64 --Ci 128 --Co 64 --K 1 --relu" "--H 64 --Ci 64 --Co 128 --K 1 --res --relu" \
             "--H 64 --Ci 64 --Co 64 --K 3 --relu" \
             "--H 32 --Ci 192 --Co 96 --K 1 --relu" "--H 32 --Ci 96 --Co 96 --K 3 --relu" \
             "--H 32 --Ci 96 --Co 192 --K 1 --res --relu" "--H 128 --Ci 128 --Co 128 --K 5 --stride 2"; do
  for m in "" --bf6; do
    python3 scripts/conv_micro.py $shape $m
  done
done
