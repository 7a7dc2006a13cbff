#!/bin/bash
# One GPU-box evidence pass, by phase: scripts/check.sh <tag> <phase>...
#   tests   full -m gpu suite           smoke  __graft_entry__.smoke()
#   tests1  the suite without the AMP-fixture test; ampfix  that test alone (its failure does not stop the pass)
#   bench   the driver's bench command  stats  rocprofv3 kernel stats of a short bench command
#   pmc     FETCH_SIZE / WRITE_SIZE passes -> HBM bytes per launch of the fp32 and AMP dominant kernels
#   steps   per-kernel tables of 10 replayed fp32 / AMP steps (scripts/profile_steps.sh)
#   mem     peak device memory with the deferred weight-gradient reduces on / off (scripts/mem_probe.py)
#   dist    the N>1 rehearsal (scripts/dist_rehearsal.sh)
#   probe   scripts/bf16x6_probe (fp32 GEMM: native f32 MFMA vs the bf16x6 split, speed and error)
#   sq      SQ-counter passes of the bf16x6 kernels in isolation (scripts/pmc_sq.sh)
#   layers  per-launch conv tables of one fp32 / AMP step (scripts/layer_table.py)
# Every step runs under its own time limit (scripts/gpu_run.sh) and the pass stops at the first crash-like exit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval"
for ph in "$@"; do
  case $ph in
    tests) scripts/gpu_run.sh "gputests:600:python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -s" || exit $? ;;
    tests1) scripts/gpu_run.sh "gputests:600:python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -s --deselect tests/test_parity_gpu.py::test_amp_matches_reference_autocast_fixture" || exit $? ;;
    ampfix) scripts/gpu_run.sh "ampfix:200:python -u -m pytest tests/test_parity_gpu.py -v --timeout 180 --timeout-method thread -m gpu -s -k test_amp_matches_reference_autocast_fixture" ;;
    smoke) scripts/gpu_run.sh "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" || exit $? ;;
    bench) scripts/gpu_run.sh "bench_full:500:python3 bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
           grep '^{' gpurun_out/bench_full.log > gpurun_out/${tag}_bench_line.json ;;
    stats) scripts/gpu_run.sh "stats:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run -- python3 $BENCH" || exit $?
           python3 scripts/prof_summary.py gpurun_out/${tag}_stats/run_kernel_stats.csv 11 > gpurun_out/${tag}_bench_summary.txt ;;
    pmc)   scripts/gpu_run.sh \
             "pmc_fetch:500:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python3 $BENCH" \
             "pmc_write:500:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python3 $BENCH" || exit $?
           for leg in fp32 amp; do
             if [ $leg = fp32 ]; then sel="d['roofline']['kernel']"; out=${tag}_pmc_traffic.json; else sel="d['amp']['roofline']['kernel']"; out=${tag}_pmc_traffic_amp.json; fi
             K=$(python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_line.json')); print($sel.split(' (')[0])") || exit 1
             python3 scripts/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write --kernel "$K" --out gpurun_out/$out \
               --command "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace --output-format csv -- python3 $BENCH" >> gpurun_out/pmc_traffic.log 2>&1
           done ;;
    steps) bash scripts/profile_steps.sh $tag || exit $? ;;
    mem)   scripts/gpu_run.sh "mem_defer1:200:python3 scripts/mem_probe.py" "mem_defer0:200:HYRES_WGRAD_DEFER=0 python3 scripts/mem_probe.py" || exit $?
           cat gpurun_out/mem_defer1.log gpurun_out/mem_defer0.log | grep WGRAD_DEFER > gpurun_out/${tag}_mem_probe.txt ;;
    dist)  bash scripts/dist_rehearsal.sh; echo "dist rehearsal exit $?" ;;
    sq)    bash scripts/pmc_sq.sh $tag || exit $? ;;
    ab)    bash scripts/ab_alt.sh $tag || exit $? ;;
    h1x1)  scripts/gpu_run.sh "h1x1:300:for s in '--H 128 --Ci 64 --Co 128 --K 1 --res --relu' '--H 128 --Ci 128 --Co 64 --K 1 --relu' '--H 64 --Ci 64 --Co 128 --K 1 --res --relu' '--H 256 --Ci 64 --Co 64 --K 1 --relu'; do for m in '' --no-stream-h; do python3 scripts/conv_micro.py --io16 \$s \$m; done; done" || exit $?
           grep "us," gpurun_out/h1x1.log > gpurun_out/${tag}_h1x1.txt ;;
    ru)    scripts/gpu_run.sh "ru_micro:200:python3 scripts/ru_micro.py && python3 scripts/ru_micro.py --H 64 --W 64" || exit $?
           grep "us," gpurun_out/ru_micro.log > gpurun_out/${tag}_ru_micro.txt ;;
    layers) scripts/gpu_run.sh "layers_fp32:200:python3 scripts/layer_table.py" "layers_amp:200:python3 scripts/layer_table.py --amp" || exit $?
           cp gpurun_out/layers_fp32.log gpurun_out/${tag}_layers_fp32.txt; cp gpurun_out/layers_amp.log gpurun_out/${tag}_layers_amp.txt ;;
    probe) scripts/gpu_run.sh "bf16x6_probe:120:scripts/bf16x6_probe" \
             "bf6_micro:300:for H in 128 256; do for m in '' --bf6; do python3 scripts/conv_micro.py --H \$H \$m; python3 scripts/conv_micro.py --H \$H --res --relu \$m; done; done" \
             "bf6_families:400:bash scripts/bf6_families.sh" || exit $?
           grep -h "us," gpurun_out/bf16x6_probe.log gpurun_out/bf6_micro.log gpurun_out/bf6_families.log > gpurun_out/${tag}_bf6_micro.txt ;;
    wgpf)  scripts/gpu_run.sh "wgpf:300:for s in '--H 128 --Ci 64 --Co 128' '--H 128 --Ci 128 --Co 64' '--H 128 --Ci 128 --Co 128' '--H 256 --Ci 64 --Co 64' '--H 256 --Ci 64 --Co 192' '--H 64 --Ci 64 --Co 128' '--H 32 --Ci 96 --Co 192' '--H 32 --Ci 640 --Co 768'; do python3 scripts/wgrad_micro.py \$s --K 1 --ab 15=1,2,1,2; done; for s in '--H 128 --Ci 64 --Co 64' '--H 256 --Ci 64 --Co 64' '--H 64 --Ci 64 --Co 64' '--H 128 --Ci 128 --Co 128' '--H 32 --Ci 96 --Co 96'; do python3 scripts/wgrad_micro.py \$s --K 3 --ab 16=1,2,1,2; done; python3 scripts/wgrad_micro.py --H 32 --Ci 192 --Co 384 --K 5 --ab 16=1,2,1,2" || exit $?
           grep -h "key1[56]" gpurun_out/wgpf.log > gpurun_out/${tag}_wgrad_pf_ab.txt ;;
    serial) scripts/gpu_run.sh "serial_fp32:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_serial -o run -- python3 scripts/step_profile.py --marker --serial --steps 10" || exit $?
           python3 scripts/prof_summary.py gpurun_out/${tag}_serial/run_kernel_trace.csv 10 > gpurun_out/${tag}_train_serial_summary.txt ;;
    pmcfam) bash scripts/pmc_families.sh $tag || exit $? ;;
    tuneab) bash scripts/tune_ab.sh $tag "default=" "nopf2=HYRES_TUNE=15=1,16=1" "nohf=HYRES_TUNE=17=0" "nofold=HYRES_FOLD_SA_MUL=0" || exit $? ;;
    repro) scripts/gpu_run.sh "repro_native_b6v:200:scripts/bf6_interference_repro 20 30 native-b6v" || exit $?
           cp gpurun_out/repro_native_b6v.log gpurun_out/${tag}_repro_native_b6v.txt ;;
    split32) scripts/gpu_run.sh "split32:400:for T in '' 1=1024 1=2048 1=4096 1=2048,2=2; do for s in '--H 32 --Ci 96 --Co 96 --K 3 --relu' '--H 32 --Ci 192 --Co 96 --K 1 --relu' '--H 32 --Ci 96 --Co 192 --K 1 --res --relu' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 64 --Ci 64 --Co 128 --K 3 --relu'; do echo \"T=\$T\"; HYRES_TUNE=\$T python3 scripts/conv_micro.py \$s --bf6; done; done; for T in '' 3=1024 3=2048 3=2048,4=2; do for s in '--H 32 --Ci 96 --Co 96 --K 3' '--H 32 --Ci 96 --Co 192 --K 1' '--H 32 --Ci 192 --Co 96 --K 1'; do echo \"T=\$T\"; HYRES_TUNE=\$T python3 scripts/wgrad_micro.py \$s; done; done" || exit $?
           grep -h "T=\|us" gpurun_out/split32.log > gpurun_out/${tag}_split32.txt ;;
    tile32) scripts/gpu_run.sh "tile32:400:for t in -1 0 1 2 3 4; do for s in '--H 32 --Ci 96 --Co 96 --K 3 --relu' '--H 32 --Ci 192 --Co 96 --K 1 --relu' '--H 32 --Ci 96 --Co 192 --K 1 --res --relu' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 64 --Ci 64 --Co 128 --K 3 --relu' '--H 32 --Ci 640 --Co 512 --K 1'; do python3 scripts/conv_micro.py \$s --bf6 --tile \$t | sed \"s/^/tile \$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/tile32.log > gpurun_out/${tag}_tile32.txt ;;
    t6)    scripts/gpu_run.sh "t6:400:python -u -m pytest tests/test_parity_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -s -k 'prelu or refine or checkerboard_masked or captured'" || exit $? ;;
    ab6)   bash scripts/tune_ab.sh $tag "default=" "noprelu=HYRES_FOLD_PRELU=0" "tile5=HYRES_TUNE=18=0" || exit $? ;;
    serialab) scripts/gpu_run.sh "serial_fold1:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_serial_f1 -o run -- python3 scripts/step_profile.py --marker --serial --steps 10" \
                "serial_fold0:300:HYRES_FOLD_PRELU=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_serial_f0 -o run -- python3 scripts/step_profile.py --marker --serial --steps 10" || exit $?
           python3 scripts/prof_summary.py gpurun_out/${tag}_serial_f1/run_kernel_trace.csv 10 > gpurun_out/${tag}_serial_fold1.txt
           python3 scripts/prof_summary.py gpurun_out/${tag}_serial_f0/run_kernel_trace.csv 10 > gpurun_out/${tag}_serial_fold0.txt ;;
    as)    scripts/gpu_run.sh \
             "as_fetch:300:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_as_f -o run -- python3 scripts/as_traffic.py" \
             "as_write:300:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${tag}_as_w -o run -- python3 scripts/as_traffic.py" || exit $?
           python3 scripts/as_traffic.py --summarize gpurun_out/${tag}_as_f gpurun_out/${tag}_as_w --out gpurun_out/${tag}_as_traffic.json ;;
    b6sw)  scripts/gpu_run.sh "b6sw:400:for t in 1 0 1 0; do for s in '--H 32 --Ci 96 --Co 96 --K 3 --relu' '--H 32 --Ci 192 --Co 96 --K 1 --relu' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 64 --Ci 64 --Co 128 --K 3 --relu' '--H 32 --Ci 640 --Co 512 --K 1' '--H 128 --Ci 128 --Co 128 --K 5 --stride 2'; do HYRES_TUNE=19=\$t python3 scripts/conv_micro.py \$s --bf6 | sed \"s/^/b6sw=\$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/b6sw.log > gpurun_out/${tag}_b6sw.txt ;;
    b6db)  scripts/gpu_run.sh "b6db:400:for t in 0 1 0 1; do for s in '--H 32 --Ci 96 --Co 96 --K 3 --relu' '--H 32 --Ci 192 --Co 96 --K 1 --relu' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 128 --Ci 128 --Co 128 --K 5 --stride 2' '--H 64 --Ci 64 --Co 128 --K 3 --relu' '--H 64 --Ci 128 --Co 128 --K 3 --relu'; do HYRES_TUNE=20=\$t python3 scripts/conv_micro.py \$s --bf6 | sed \"s/^/b6db=\$t /\"; done; done" \
             "b6dbtest:300:python -u -m pytest tests/test_bf6_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k staging" || exit $?
           grep -h "us" gpurun_out/b6db.log > gpurun_out/${tag}_b6db.txt ;;
    tb6)   scripts/gpu_run.sh "tb6:500:python -u -m pytest tests/test_bf6_gpu.py tests/test_coresidency_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu" || exit $? ;;
    ab7)   bash scripts/tune_ab.sh $tag "default=" "nodb=HYRES_TUNE=20=0" || exit $? ;;
    tile5) scripts/gpu_run.sh "tile5:400:for t in -1 0 1 3 4; do for s in '--H 128 --Ci 128 --Co 128 --K 5 --stride 2' '--H 64 --Ci 128 --Co 192 --K 5 --stride 2' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 64 --Ci 128 --Co 128 --K 3 --relu' '--H 32 --Ci 192 --Co 384 --K 3'; do python3 scripts/conv_micro.py \$s --bf6 --tile \$t | sed \"s/^/tile \$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/tile5.log > gpurun_out/${tag}_tile5.txt ;;
    tile6) scripts/gpu_run.sh "tile6:400:for t in 1 0 1 0; do for s in '--H 128 --Ci 128 --Co 128 --K 5 --stride 2' '--H 64 --Ci 128 --Co 192 --K 5 --stride 2' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 32 --Ci 96 --Co 192 --K 1 --res --relu' '--H 32 --Ci 640 --Co 512 --K 1'; do HYRES_TUNE=18=\$t python3 scripts/conv_micro.py \$s --bf6 | sed \"s/^/rule18=\$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/tile6.log > gpurun_out/${tag}_tile6.txt
           bash scripts/tune_ab.sh $tag "default=" "r5tile=HYRES_TUNE=18=0" || exit $? ;;
    tile1x1) scripts/gpu_run.sh "tile1x1:400:for t in -1 0 1 2 3 4; do for s in '--H 256 --Ci 64 --Co 192 --K 1' '--H 256 --Ci 192 --Co 64 --K 1 --relu' '--H 128 --Ci 128 --Co 128 --K 1' '--H 128 --Ci 128 --Co 128 --K 1 --relu'; do python3 scripts/conv_micro.py \$s --bf6 --tile \$t | sed \"s/^/tile \$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/tile1x1.log > gpurun_out/${tag}_tile1x1.txt ;;
    sab)   scripts/gpu_run.sh "sabtest:300:python -u -m pytest tests/test_stream_b6_gpu.py tests/test_parity_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -k 'sa_bwd or sa_fold or c2_size'" \
             "sabmicro:300:for t in 1 0 1 0; do HYRES_TUNE=21=\$t python3 scripts/layer_table.py > gpurun_out/sab_layers_\$t.txt 2>&1 && grep 'epi6' gpurun_out/sab_layers_\$t.txt | sed \"s/^/sab=\$t /\"; done" || exit $?
           grep -h "sab=" gpurun_out/sabmicro.log > gpurun_out/${tag}_sab.txt
           bash scripts/tune_ab.sh $tag "default=" "nosab=HYRES_TUNE=21=0" || exit $? ;;
    ab8)   bash scripts/tune_ab.sh $tag "default=" "nodefer=HYRES_DEFER_ON_GRAD=0" || exit $? ;;
    ab9)   scripts/gpu_run.sh "t9:300:python -u -m pytest tests/test_parity_gpu.py tests/test_amp_f16_act_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -k 'attn_gate or train or c2_size or attention or residual_unit'" || exit $?
           bash scripts/serial_one.sh $tag || exit $? ;;
    wg5)   scripts/gpu_run.sh "wg5test:300:python -u -m pytest tests/test_bf6_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -k prefetch2" \
             "wg5:300:for s in '--H 128 --Ci 128 --Co 128 --K 5 --stride 2' '--H 64 --Ci 128 --Co 192 --K 5 --stride 2' '--H 32 --Ci 192 --Co 384 --K 5' '--H 16 --Ci 192 --Co 128 --K 5 --stride 2'; do python3 scripts/wgrad_micro.py \$s --ab 22=0,1,0,1; done" || exit $?
           grep -h "key22" gpurun_out/wg5.log > gpurun_out/${tag}_wg5.txt
           bash scripts/tune_ab.sh $tag "default=" "nowg5=HYRES_TUNE=22=0" || exit $? ;;
    tiledc) scripts/gpu_run.sh "tiledc:400:for t in -1 0 1 3 4; do for s in '--H 64 --Ci 128 --Co 128 --deconv' '--H 32 --Ci 192 --Co 128 --deconv' '--H 16 --Ci 128 --Co 128 --deconv' '--H 8 --Ci 128 --Co 128 --deconv'; do python3 scripts/conv_micro.py \$s --bf6 --tile \$t | sed \"s/^/tile \$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/tiledc.log > gpurun_out/${tag}_tiledc.txt ;;
    thinpmc) bash scripts/pmc_families.sh $tag thin || exit $? ;;
    thin)  scripts/gpu_run.sh "thintest:300:python -u -m pytest tests/test_bf6_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -k thin_window" \
             "thinmicro:300:for s in '--H 256 --Ci 3 --Co 64 --K 3' '--H 256 --Ci 64 --Co 3 --K 3' '--H 256 --Ci 3 --Co 128 --K 5 --stride 2'; do python3 scripts/wgrad_micro.py \$s --ab 23=0,1,0,1; done" || exit $?
           grep -h "key23" gpurun_out/thinmicro.log > gpurun_out/${tag}_thin.txt ;;
    serialamp) bash scripts/serial_one.sh ${tag}amp --amp || exit $? ;;
    tileh) scripts/gpu_run.sh "tileh:400:for t in -1 0 1 3 4; do for s in '--H 32 --Ci 96 --Co 96 --K 3 --relu' '--H 32 --Ci 192 --Co 96 --K 1 --relu' '--H 32 --Ci 96 --Co 192 --K 1 --res --relu' '--H 32 --Ci 384 --Co 192 --K 3 --relu' '--H 32 --Ci 640 --Co 512 --K 1' '--H 64 --Ci 128 --Co 192 --K 5 --stride 2'; do python3 scripts/conv_micro.py \$s --f16 --tile \$t | sed \"s/^/tile \$t /\"; done; done" || exit $?
           grep -h "us" gpurun_out/tileh.log > gpurun_out/${tag}_tileh.txt ;;
    ab10)  bash scripts/tune_ab.sh $tag "default=" "split128=HYRES_TUNE=6=128" "split192=HYRES_TUNE=6=192" || exit $? ;;
    gate)  scripts/gpu_run.sh "gate:200:python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -s -k 'attn_gate or amp or sa_fold or stream_hf or refine or prelu or bilinear'" || exit $? ;;
    rs)    scripts/gpu_run.sh "rstest:300:python -u -m pytest tests/test_stream_b6_gpu.py tests/test_parity_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -k 'rowscale or sa_bwd or sa_fold or c2_size'" || exit $?
           bash scripts/serial_one.sh $tag || exit $? ;;
    ab11)  bash scripts/tune_ab.sh $tag "default=" "nosa21=HYRES_TUNE=21=0" || exit $? ;;
    s128)  scripts/gpu_run.sh "s128test:300:python -u -m pytest tests/test_stream_b6_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu -k 'matches_fp64'" \
             "s128:300:for r in 1 2; do for m in '' '--mask' '--relu'; do for o in '' '--no-stream-b6'; do python3 scripts/conv_micro.py --H 128 --Ci 128 --Co 128 --K 1 --bf6 \$m \$o | sed \"s/^/[\$m \$o] /\"; done; done; done" || exit $?
           grep -h "us" gpurun_out/s128.log > gpurun_out/${tag}_s128.txt ;;
    ab12)  bash scripts/tune_ab.sh $tag "default=" "nofold=HYRES_FOLD_PRELU=0" || exit $? ;;
    *) echo "unknown phase $ph"; exit 2 ;;
  esac
done
