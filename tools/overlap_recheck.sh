set -o pipefail
mkdir -p gpurun_out/s16
for r in 1 2; do for ov in 3,3,1 3,3,2 3,4,1 3,2,1 4,3,1; do
  timeout -k 10 200 python bench.py --overlap $ov --cpu-seconds 0 --serial-steps 0 --steps 50 > gpurun_out/s16/ov_${ov}_$r.json 2>/dev/null || { echo "FAILED $ov"; exit 1; }
  python -c "import json;j=json.loads(open('gpurun_out/s16/ov_${ov}_$r.json').read().strip().splitlines()[-1]);print($r,'$ov',round(j['value']),round(j['ms_per_step'],4),j['verified'])"
done; done
