#!/bin/bash
# One GPU session on the box: the steps named on the command line, in order, each under its own
# time limit, stopping at the first failure.
# usage: tools/session.sh TAG step [step ...]
#   steps: tests (pytest -m gpu), smoke, bench (default headline line), prof (rocprofv3 kernel
#          stats of a short headline run), dropin (drop-in line), pmc (HBM fetch/write passes),
#          k=<pytest -k expr> (a subset of the GPU tests), counters (kernel trace + PMC passes,
#          tools/prof_counters.sh), workloads (the side-row benches: euroc, reloc, tri, bf, kfdb,
#          tum, host-io), ab (tools/variants.py run: the headline per built variant),
#          frame_trace (kernel + API trace of the one-call Frame, K = 1 and 8)
# Copy what is kept into profiles/ with tools/collect_profiles.sh.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
        || { echo "GPU TESTS FAILED"; tail -40 $OUT/pytest_gpu.log; exit 1; }
      tail -1 $OUT/pytest_gpu.log ;;
    k=*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${step#k=}" > $OUT/pytest_k.log 2>&1 \
        || { echo "GPU TESTS (-k) FAILED"; tail -40 $OUT/pytest_k.log; exit 1; }
      tail -3 $OUT/pytest_k.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
        || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
      python -c "import json,sys; j=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', j['value'], j['ms_per_step'], json.dumps(j.get('roofline'))[:400])" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --serial-steps 0 --no-kernel-timing > $OUT/prof.log 2>&1 \
        || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
      echo prof done ;;
    dropin)
      timeout -k 10 600 python bench.py --workload dropin --frames 300 > $OUT/dropin.json 2> $OUT/dropin.err \
        || { echo "DROPIN BENCH FAILED"; tail -20 $OUT/dropin.err; exit 1; }
      echo dropin done ;;
    counters)
      timeout -k 10 900 bash tools/prof_counters.sh $OUT/prof --steps 10 --warmup 3 > $OUT/counters.log 2>&1 \
        || { echo "COUNTERS FAILED"; tail -20 $OUT/counters.log; exit 1; }
      echo counters done ;;
    counters_euroc)
      timeout -k 10 900 bash tools/prof_counters.sh $OUT/prof_euroc --workload euroc --steps 10 --warmup 3 > $OUT/counters_euroc.log 2>&1 \
        || { echo "EUROC COUNTERS FAILED"; tail -20 $OUT/counters_euroc.log; exit 1; }
      echo euroc counters done ;;
    counters_match)
      # FETCH_SIZE and WRITE_SIZE passes (one counter per run) of the matcher workloads; the bf
      # run times both distance kernels (k_bf_mfma, then k_bf_top2 as alt_kernel)
      for w in bf reloc triangulation; do
        for c in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/pmc_${w}_${c}dir -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/pmc_${w}_$c.log 2>&1 \
            || { echo "PMC $w $c FAILED"; tail -20 $OUT/pmc_${w}_$c.log; exit 1; }
          cp $OUT/pmc_${w}_${c}dir/run_counter_collection.csv $OUT/pmc_${w}_$c.csv
        done
        timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/trace_$w.log 2>&1 \
          || { echo "TRACE $w FAILED"; tail -20 $OUT/trace_$w.log; exit 1; }
      done
      echo match counters done ;;
    workloads)
      for w in euroc reloc triangulation bf kfdb tum; do
        timeout -k 10 300 python bench.py --workload $w --cpu-seconds 5 > $OUT/$w.json 2> $OUT/$w.err \
          || { echo "WORKLOAD $w FAILED"; tail -20 $OUT/$w.err; exit 1; }
      done
      timeout -k 10 300 python bench.py --host-io --cpu-seconds 0 > $OUT/hostio.json 2> $OUT/hostio.err \
        || { echo "HOST-IO FAILED"; tail -20 $OUT/hostio.err; exit 1; }
      echo workloads done ;;
    ab)
      timeout -k 10 900 python tools/variants.py run --rounds 2 > $OUT/ab.txt 2>&1 \
        || { echo "AB FAILED"; tail -5 $OUT/ab.txt; exit 1; }
      cat $OUT/ab.txt ;;
    frame_trace)
      bash tools/frame_trace.sh ${OUT#gpurun_out/}/tr || exit 1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
