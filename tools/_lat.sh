export TMPDIR=/tmp
mkdir -p gpurun_out/lat
for B in 1 4 16 64; do
timeout -k 10 120 python bench.py --batch $B --distinct 1 --cpu-seconds 0 --no-kernel-timing --steps 200 --warmup 20 > gpurun_out/lat/b$B.json 2> gpurun_out/lat/b$B.err || { tail gpurun_out/lat/b$B.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/lat/b$B.json'));print($B, j['ms_per_step'], j['value'])"
done
timeout -k 10 120 python bench.py --batch 1 --distinct 1 --cpu-seconds 0 --no-kernel-timing --steps 200 --warmup 20 --host-io > gpurun_out/lat/b1h.json 2> gpurun_out/lat/b1h.err || { tail gpurun_out/lat/b1h.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/lat/b1h.json'));print('hostio', j['ms_per_step'], j['value'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lat/prof -o run --output-format csv -- python3 bench.py --batch 1 --distinct 1 --cpu-seconds 0 --no-kernel-timing --steps 20 --warmup 2 > gpurun_out/lat/prof.log 2>&1 || exit 1
cat gpurun_out/lat/prof/run_kernel_stats.csv | cut -c1-160
