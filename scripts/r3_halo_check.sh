cd "$GRAFT_REPO_ROOT"
scripts/gpu_run.sh \
 "ddp:300:python -u -m pytest tests/test_ddp_gpu.py -v -s --timeout 250 --timeout-method thread -m gpu" \
 "amp:400:python -u -m pytest tests/test_parity_gpu.py tests/test_vgg.py -v -s --timeout 200 --timeout-method thread -m gpu -k 'amp or fp16_activation or c5_fp16 or vgg'" \
 "f16micro:200:python scripts/conv_micro.py --f16 && python scripts/conv_micro.py --f16 --H 256 && python scripts/conv_micro.py --f16 --H 64 --Ci 128 --Co 128 && HYRES_CONV_HALO16=0 python scripts/conv_micro.py --f16 && HYRES_CONV_HALO16=0 python scripts/conv_micro.py --f16 --H 256"
