#!/bin/bash
# C3 at the driver's flags for several pre-warm lengths, twice each.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for pw in 30 150 500 1000; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --prewarm-ms $pw > gpurun_out/pab_$pw.out 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/pab_$pw.out').read().strip().splitlines()[-1]);print('pw=$pw',d['value'],d['ms_per_step'],d['prewarm'])"
done; done
