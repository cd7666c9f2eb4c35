export TMPDIR=/tmp
mkdir -p gpurun_out/lat2
for TH in 64 32 16 8; do
for B in 1 8; do
ORBX_STRIP_TH="$TH,$TH,$TH,$TH,$TH,$TH,$TH,$TH" timeout -k 10 120 python bench.py --batch $B --distinct 1 --cpu-seconds 0 --steps 200 --warmup 20 > gpurun_out/lat2/t$TH-b$B.json 2> gpurun_out/lat2/t$TH-b$B.err || { tail gpurun_out/lat2/t$TH-b$B.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/lat2/t$TH-b$B.json'));print($TH, $B, round(j['ms_per_step'],4), j['mean_stereo_matches'], j['roofline']['kernel_ms_per_step'])"
done
done
