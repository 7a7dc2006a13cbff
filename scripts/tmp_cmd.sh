#!/bin/bash
scripts/gpu_run.sh "gpu_tests:800:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" && scripts/profile_round.sh r2v3 && scripts/profile_steps.sh r2v3
