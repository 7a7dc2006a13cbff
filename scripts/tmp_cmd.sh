#!/bin/bash
scripts/gpu_run.sh "bench_full:420:python3 bench.py"
