#!/bin/bash
# Round-4 measurement session: GPU tests, the headline's kernel trace and PMC passes, then every
# bench line.  usage: tools/gpu_session_final_r4.sh TAG [skip-tests]
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
fi
bash tools/prof_counters.sh $OUT/prof || { echo "PROFILING FAILED"; exit 1; }
F=$(ls $OUT/prof/pmc3/*counter_collection.csv | head -1)
W=$(ls $OUT/prof/pmc4/*counter_collection.csv | head -1)
I=$(ls $OUT/prof/pmc1/*counter_collection.csv | head -1)
V=$(ls $OUT/prof/pmc5/*counter_collection.csv | head -1)
timeout -k 10 600 python bench.py --traffic-csv "$F,$W" --insts-csv "$I,$V" > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('headline',round(d['value']),d['ms_per_step'],d['verified'],r['kernel'],round(r['frac'],4),r['avg_launch_ms'])"
bash tools/prof_counters.sh $OUT/prof_euroc --workload euroc || { echo "EUROC PROFILING FAILED"; exit 1; }
FE=$(ls $OUT/prof_euroc/pmc3/*counter_collection.csv | head -1)
WE=$(ls $OUT/prof_euroc/pmc4/*counter_collection.csv | head -1)
IE=$(ls $OUT/prof_euroc/pmc1/*counter_collection.csv | head -1)
VE=$(ls $OUT/prof_euroc/pmc5/*counter_collection.csv | head -1)
timeout -k 10 600 python bench.py --workload euroc --traffic-csv "$FE,$WE" --insts-csv "$IE,$VE" > $OUT/euroc.json 2> $OUT/euroc.err || { echo "EUROC BENCH FAILED"; tail -20 $OUT/euroc.err; exit 1; }
timeout -k 10 600 python bench.py --workload reloc --steps 10 --warmup 2 > $OUT/reloc.json 2> $OUT/reloc.err || { echo "RELOC BENCH FAILED"; tail -20 $OUT/reloc.err; exit 1; }
timeout -k 10 600 python bench.py --workload triangulation --steps 20 --warmup 3 > $OUT/tri.json 2> $OUT/tri.err || { echo "TRI BENCH FAILED"; tail -20 $OUT/tri.err; exit 1; }
timeout -k 10 600 python bench.py --workload dropin --frames 300 > $OUT/dropin.json 2> $OUT/dropin.err || { echo "DROPIN BENCH FAILED"; tail -20 $OUT/dropin.err; exit 1; }
timeout -k 10 600 python bench.py --workload kfdb --steps 200 --warmup 10 > $OUT/kfdb.json 2> $OUT/kfdb.err || { echo "KFDB BENCH FAILED"; tail -20 $OUT/kfdb.err; exit 1; }
timeout -k 10 600 python bench.py --workload bf --steps 20 --warmup 3 > $OUT/bf.json 2> $OUT/bf.err || { echo "BF BENCH FAILED"; tail -20 $OUT/bf.err; exit 1; }
timeout -k 10 600 python bench.py --workload tum --frames 300 > $OUT/tum.json 2> $OUT/tum.err || { echo "TUM BENCH FAILED"; tail -20 $OUT/tum.err; exit 1; }
timeout -k 10 300 python bench.py --host-io --steps 20 --warmup 4 --cpu-seconds 0 > $OUT/hostio.json 2> $OUT/hostio.err || { echo "HOSTIO BENCH FAILED"; tail -20 $OUT/hostio.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_reloc -o run --output-format csv -- python3 bench.py --workload reloc --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/prof_reloc.log 2>&1 || { echo "RELOC TRACE FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_tri -o run --output-format csv -- python3 bench.py --workload triangulation --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/prof_tri.log 2>&1 || { echo "TRI TRACE FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bf -o run --output-format csv -- python3 bench.py --workload bf --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/prof_bf.log 2>&1 || { echo "BF TRACE FAILED"; exit 1; }
python tools/dropin_data.py /tmp/dd 8 > /dev/null && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_dropin -o run --output-format csv -- tests/native/facade_test bench /tmp/dd 100 20 1 frame > $OUT/prof_dropin.log 2>&1 || { echo "DROPIN TRACE FAILED"; exit 1; }
python tools/dropin_data.py /tmp/dd 8 > /dev/null && timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd 1,8 > $OUT/dropin_ab.txt 2>&1 || { echo "DROPIN AB FAILED"; tail -5 $OUT/dropin_ab.txt; exit 1; }
cat $OUT/dropin_ab.txt
echo session done
