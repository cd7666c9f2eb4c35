# headline at several batch sizes / in-flight counts (timed schedule only).  usage: TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
for cfg in "512 2" "768 2" "1024 2" "1024 1"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --batch $1 --inflight $2 --steps 30 --warmup 5 --cpu-seconds 0 --serial-steps 0 > $O/b$1_i$2_$rep.json 2> $O/b$1_i$2_$rep.err || { tail -5 $O/b$1_i$2_$rep.err; exit 1; }
  python3 -c "
import json; j=json.loads(open('$O/b$1_i$2_$rep.json').read().strip().splitlines()[-1])
print('$rep B=$1 inflight=$2', round(j['value']), round(j['ms_per_step'],3), j['verified'])"
done; done
