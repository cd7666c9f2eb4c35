#!/bin/bash
# Drop-in line (bench.py --workload dropin) of each A/B variant of tools/_variants.json,
# interleaved over two rounds; prints K -> median ms / pairs/s per variant.
# usage: tools/dropin_variants.sh OUTDIR
set -o pipefail
OUT=$1; mkdir -p $OUT
for rep in 1 2; do
  for name in $(python3 -c "import json; print(' '.join(json.load(open('tools/_variants.json'))))"); do
    lib=$(python3 -c "import json; print(json.load(open('tools/_variants.json'))['$name']['lib'])")
    ORBX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload dropin --frames 300 --cpu-seconds 0 > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.err \
      || { echo "FAILED $name"; tail -5 $OUT/${name}_$rep.err; exit 1; }
    python3 -c "
import json; j=json.loads(open('$OUT/${name}_$rep.json').read().strip().splitlines()[-1])
print('$name', $rep, ' '.join(f\"K{t['trackers']}={t['latency']['median_ms']:.4f}ms/{t['pairs_per_s']:.0f}\" for t in j['per_trackers']))"
  done
done
