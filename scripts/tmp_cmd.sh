#!/bin/bash
scripts/gpu_run.sh "t_engine:500:python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread"
