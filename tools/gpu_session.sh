#!/bin/bash
# One GPU session: GPU tests, kernel trace + PMC passes, then the bench lines with the CPU
# baselines and the measured traffic.  usage: tools/gpu_session.sh TAG
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
bash tools/prof_counters.sh $OUT/prof || { echo "PROFILING FAILED"; exit 1; }
F=$(ls $OUT/prof/pmc3/*counter_collection.csv 2>/dev/null | head -1)
W=$(ls $OUT/prof/pmc4/*counter_collection.csv 2>/dev/null | head -1)
echo "pmc: $F $W"
timeout -k 10 600 python bench.py --traffic-csv "$F,$W" > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
# EuRoC mono tracking workload (configs[2]): trace + traffic passes, then its bench line
bash tools/prof_counters.sh $OUT/prof_euroc --workload euroc || { echo "EUROC PROFILING FAILED"; exit 1; }
FE=$(ls $OUT/prof_euroc/pmc3/*counter_collection.csv 2>/dev/null | head -1)
WE=$(ls $OUT/prof_euroc/pmc4/*counter_collection.csv 2>/dev/null | head -1)
timeout -k 10 600 python bench.py --workload euroc --traffic-csv "$FE,$WE" > $OUT/euroc.json 2> $OUT/euroc.err || { echo "EUROC BENCH FAILED"; tail -20 $OUT/euroc.err; exit 1; }
cat $OUT/euroc.json
timeout -k 10 600 python bench.py --workload reloc --steps 10 --warmup 2 > $OUT/reloc.json 2> $OUT/reloc.err || { echo "RELOC BENCH FAILED"; tail -20 $OUT/reloc.err; exit 1; }
cat $OUT/reloc.json
timeout -k 10 600 python bench.py --workload triangulation --steps 20 --warmup 3 > $OUT/tri.json 2> $OUT/tri.err || { echo "TRI BENCH FAILED"; tail -20 $OUT/tri.err; exit 1; }
cat $OUT/tri.json
# kernel traces of the matcher workloads (configs[3], configs[4])
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_reloc -o run --output-format csv -- python3 bench.py --workload reloc --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/prof_reloc.log 2>&1 || { echo "RELOC TRACE FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_tri -o run --output-format csv -- python3 bench.py --workload triangulation --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/prof_tri.log 2>&1 || { echo "TRI TRACE FAILED"; exit 1; }
echo session done
