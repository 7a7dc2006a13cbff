cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
 "f16micro:200:python scripts/conv_micro.py --f16 && python scripts/conv_micro.py --f16 --H 256 && python scripts/conv_micro.py --f16 --H 64 && python scripts/conv_micro.py --f16 --res --relu && HYRES_CONV_WRES16=0 python scripts/conv_micro.py --f16 --res --relu && python scripts/conv_micro.py --f16 --Ci 128 --Co 128 --K 1" \
 "amp:400:python -u -m pytest tests/test_parity_gpu.py -v -s --timeout 200 --timeout-method thread -m gpu -k 'amp_fwd_bwd or fp16_activation or amp_train or amp_matches'"
