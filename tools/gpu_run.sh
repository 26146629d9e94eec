#!/bin/bash
# Dev tool: one GPU session on the gpurun box, logs under gpurun_out/$1.
#   STEPS="tests bench c4 c5 prof"  (any subset, in this order)
#   TESTS="tests/..."                 pytest selection (default: all -m gpu)
# Every GPU step has its own time limit; the first failure ends the call.
export TMPDIR=/tmp
O=gpurun_out/${1:-run}
mkdir -p $O
STEPS=${STEPS:-"tests bench"}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 900 --timeout-method thread \
        > $O/t_gpu.log 2>&1 || { tail -40 $O/t_gpu.log; exit 1; }
      tail -3 $O/t_gpu.log ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
      cut -c1-600 $O/bench.json ;;
    gridprof)   # grid build kernel split, headline and c5 (GCONFIGS)
      for c in ${GCONFIGS:-headline c5}; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/grid_$c -o run -- \
          python tools/grid_bench.py --config $c --no-oracle --reps 10 > $O/grid_$c.json 2> $O/grid_$c.err \
          || { tail -20 $O/grid_$c.err; exit 1; }
        cat $O/grid_$c.json
      done ;;
    query)   # query stage per config (QCONFIGS), plain timing then a kernel-stats pass
      for c in ${QCONFIGS:-headline c5}; do
        timeout -k 10 300 python tools/query_bench.py --config $c --reps 10 > $O/query_$c.json 2> $O/query_$c.err \
          || { tail -20 $O/query_$c.err; exit 1; }
        python -c "import json; d=json.load(open('$O/query_$c.json')); print('$c', [(x['query_ms'], x['frac_hbm'], x['pidx_checksum']) for x in d['cams']])"
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/qstats_$c -o run -- \
          python tools/query_bench.py --config $c --reps 3 > /dev/null 2> $O/qstats_$c.err || { tail -20 $O/qstats_$c.err; exit 1; }
      done ;;
    knnstats)   # layer statistics of the generic KNN walk (tools/_var/libpnr_qstats.so)
      PNR_LIB=$PWD/tools/_var/libpnr_qstats.so timeout -k 10 300 python tools/knn_stats.py --config ${KCONFIG:-c5} \
        > $O/knnstats.json 2> $O/knnstats.err || { tail -20 $O/knnstats.err; exit 1; }
      cat $O/knnstats.json ;;
    qpmc)   # query kernel stats + PMC passes (tools/prof_query.sh), QCONFIG
      bash tools/prof_query.sh $(basename $O)/qpmc || exit 1
      python tools/pmc_fold.py $O/qpmc k_knn k_march > $O/qpmc_fold.json; cat $O/qpmc_fold.json | head -60 ;;
    abvar)   # A/B: product libpnr vs tools/_var/libpnr_$VAR.so on tools/agg_bench.py (AB_ARGS), two rounds
      for rnd in 1 2; do for L in pointnerf_amd/libpnr.so tools/_var/libpnr_${VAR}.so; do
        PNR_LIB=$PWD/$L timeout -k 10 300 python tools/agg_bench.py $AB_ARGS >> $O/ab.jsonl 2>> $O/ab.err \
          || { tail -20 $O/ab.err; exit 1; }
      done; done
      python -c "import json; [print(d['lib'][-28:], d['stages_ms'], d['checksum']) for d in map(json.loads, open('$O/ab.jsonl'))]" ;;
    adamab)   # A/B of Adam variants: product libpnr vs tools/_var/libpnr_$VAR.so on tools/adam_bench.py, two rounds
      for rnd in 1 2; do for L in pointnerf_amd/libpnr.so tools/_var/libpnr_${VAR}.so; do
        PNR_LIB=$PWD/$L timeout -k 10 120 python tools/adam_bench.py >> $O/adam.jsonl 2>> $O/adam.err \
          || { tail -20 $O/adam.err; exit 1; }
      done; done
      cat $O/adam.jsonl ;;
    launch)   # bench.py --gpus 2 self-launch rehearsal: two ranks on the box's one GPU over gloo
      PNR_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/launch2.json \
        2> $O/launch2.err || { tail -20 $O/launch2.err; exit 1; }
      cut -c1-700 $O/launch2.json ;;
    c4|c5)
      timeout -k 10 600 python bench.py --config $s --steps 5 --warmup 2 > $O/bench_$s.json 2> $O/bench_$s.err \
        || { tail -20 $O/bench_$s.err; exit 1; }
      timeout -k 10 600 python bench.py --config $s --steps 3 --warmup 1 --emulate-world 8 --no-cpu-baseline \
        > $O/bench_${s}_ew8.json 2> $O/bench_${s}_ew8.err || { tail -20 $O/bench_${s}_ew8.err; exit 1; }
      cut -c1-400 $O/bench_$s.json ;;
    nr)
      timeout -k 10 300 python tools/nr_bench.py > $O/nr.json 2> $O/nr.err || { tail -20 $O/nr.err; exit 1; }
      cat $O/nr.json
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nrstats -o run -- \
        python tools/nr_bench.py > $O/nrstats.log 2>&1 || { tail -20 $O/nrstats.log; exit 1; } ;;
    tnew)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_neural_render.py tests/test_gpu_pack.py tests/test_gpu_backward.py \
        -m gpu -x -v --timeout 300 --timeout-method thread > $O/t_new.log 2>&1 || { tail -40 $O/t_new.log; exit 1; }
      tail -3 $O/t_new.log ;;
    train)
      timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 > $O/train.json 2> $O/train.err \
        || { tail -20 $O/train.err; exit 1; }
      timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 --train-precision fp32x3 > $O/train_x3.json \
        2> $O/train_x3.err || { tail -20 $O/train_x3.err; exit 1; }
      cut -c1-400 $O/train.json $O/train_x3.json
      python -c "import json; [print(f, {k: d.get(k) for k in ('ms_per_step', 'host_issue_ms_per_step', 'host_phase_ms_per_step')}) for f in ('$O/train.json', '$O/train_x3.json') for d in [json.loads(open(f).read().strip().splitlines()[-1])]]" ;;
    trainhost)   # host-side profile of the training step (cProfile; the step is bound by its host issue)
      timeout -k 10 300 python -m cProfile -o $O/train.prof bench.py --mode train --steps 30 --warmup 5 \
        --train-precision ${TP:-fp32h2} > $O/trainhost.json 2> $O/trainhost.err || { tail -20 $O/trainhost.err; exit 1; }
      python -c "import pstats; s = pstats.Stats('$O/train.prof'); s.sort_stats('tottime').print_stats(45); s.sort_stats('cumtime').print_stats(60)" > $O/trainhost.txt
      head -70 $O/trainhost.txt ;;
    trainprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trstats -o run -- \
        python bench.py --mode train --steps 20 --warmup 3 --train-precision ${TP:-fp32h2} > $O/trstats.log 2>&1 || { tail -20 $O/trstats.log; exit 1; } ;;
    trainab)   # training-step variants: product libpnr vs tools/_var/libpnr_t*.so (bench line + kernel stats each)
      for L in pointnerf_amd/libpnr.so tools/_var/libpnr_t*.so; do
        n=$(basename $L .so)
        PNR_LIB=$PWD/$L timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 > $O/tab_$n.json \
          2> $O/tab_$n.err || { tail -20 $O/tab_$n.err; exit 1; }
        PNR_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tabst_$n -o run -- \
          python bench.py --mode train --steps 20 --warmup 3 > $O/tabst_$n.log 2>&1 || { tail -20 $O/tabst_$n.log; exit 1; }
        echo $n $(python -c "import json; print(json.loads(open('$O/tab_$n.json').read().strip().splitlines()[-1])['ms_per_step'])")
      done ;;
    nrab)   # the 2-D renderer tile-shape variants in tools/_var (built on the CPU side)
      for v in tools/_var/libpnr_*.so; do
        PNR_LIB=$PWD/$v timeout -k 10 200 python tools/nr_bench.py > $O/nrab_$(basename $v .so).json 2>> $O/nrab.err \
          || { tail -20 $O/nrab.err; exit 1; }
        echo $v; cat $O/nrab_$(basename $v .so).json
      done ;;
    dbg)
      timeout -k 10 200 python tools/_var/dbg_h2_train.py > $O/dbg.log 2>&1 || { tail -30 $O/dbg.log; exit 1; }
      cat $O/dbg.log ;;
    compab)   # composite rows-in-flight variants (tools/_var), two rounds
      for rnd in 1 2; do for v in tools/_var/libpnr_comp*.so; do
        PNR_LIB=$PWD/$v timeout -k 10 200 python tools/agg_bench.py --precision fp32h2 --reps 5 >> $O/compab.jsonl 2>> $O/compab.err \
          || { tail -20 $O/compab.err; exit 1; }
      done; done
      python -c "import json; [print(d['lib'][-20:], d['stages_ms'], d['checksum']) for d in map(json.loads, open('$O/compab.jsonl'))]" ;;
    qab)   # query-stage variants (tools/_var/libpnr_q*.so), two rounds
      for rnd in 1 2; do for v in tools/_var/libpnr_q*.so; do
        PNR_LIB=$PWD/$v timeout -k 10 200 python tools/query_bench.py $QAB_ARGS >> $O/qab.jsonl 2>> $O/qab.err \
          || { tail -20 $O/qab.err; exit 1; }
      done; done
      python -c "import json; [print(d['lib'][-12:], [c['query_ms'] for c in d['cams']], [c['pidx_checksum'] for c in d['cams']]) for d in map(json.loads, open('$O/qab.jsonl'))]" ;;
    gab)   # weight-gradient GEMM variants (tools/_var/libpnr_g*.so) on tools/gemm_bench.py
      for v in tools/_var/libpnr_g*.so; do
        PNR_LIB=$PWD/$v timeout -k 10 120 python tools/gemm_bench.py >> $O/gab.jsonl 2>> $O/gab.err \
          || { tail -20 $O/gab.err; exit 1; }
      done
      cat $O/gab.jsonl ;;
    tnr)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_neural_render.py -m gpu -x -v --timeout 120 \
        --timeout-method thread > $O/t_nr.log 2>&1 || { tail -40 $O/t_nr.log; exit 1; }
      tail -3 $O/t_nr.log ;;
    benchprof)   # bench line + kernel stats + PMC passes (tools/prof_bench.sh), folded by tools/profile_summary.py
      bash tools/prof_bench.sh $(basename $O)/bp || { tail -20 $O/bp/*.log; exit 1; } ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
        python bench.py --no-cpu-baseline > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; } ;;
  esac
done
