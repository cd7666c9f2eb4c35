export TMPDIR=/tmp
mkdir -p gpurun_out/s8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s8/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 gpurun_out/s8/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s8/pytest_gpu.log
for B in 1 8 64; do
timeout -k 10 120 python bench.py --batch $B --distinct 1 --cpu-seconds 0 --steps 200 --warmup 20 > gpurun_out/s8/b$B.json 2> gpurun_out/s8/b$B.err || { tail gpurun_out/s8/b$B.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/s8/b$B.json'));print($B, round(j['ms_per_step'],4), j['mean_stereo_matches'], j['roofline']['kernel_ms_per_step'])"
done
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/s8/b512.json 2> gpurun_out/s8/b512.err || { tail gpurun_out/s8/b512.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/s8/b512.json'));print(512, j['value'], round(j['ms_per_step'],4), j['roofline']['kernel_ms_per_step'])"
timeout -k 10 300 python bench.py --workload euroc --cpu-seconds 0 > gpurun_out/s8/euroc.json 2> gpurun_out/s8/euroc.err || { tail gpurun_out/s8/euroc.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/s8/euroc.json'));print('euroc', j['value'], round(j['ms_per_step'],4), j['roofline'].get('kernel_ms_per_step'))"
