#!/bin/bash
# The hot conv geometries of the C2 step, forward with fused epilogue (scripts/conv_micro.py).
python scripts/conv_micro.py && \
python scripts/conv_micro.py --Ci 128 --Co 128 --K 1 && \
python scripts/conv_micro.py --Ci 128 --Co 64 --K 1 && \
python scripts/conv_micro.py --Ci 64 --Co 128 --K 1 && \
python scripts/conv_micro.py --Ci 128 --Co 128 --K 5 --stride 2 && \
python scripts/conv_micro.py --H 256 --Ci 64 --Co 64 && \
python scripts/conv_micro.py --H 32 --Ci 192 --Co 384 --K 3 && \
python scripts/conv_micro.py --H 256 --Ci 192 --Co 64 --K 1
