#!/bin/bash
# C3 at the driver's flags (with the pre-warm) for 2, 3 and 4 nnet streams, twice each.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for nb in 2 3 4; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --back-streams $nb > gpurun_out/sab_$nb.out 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/sab_$nb.out').read().strip().splitlines()[-1]);print('nb=$nb',d['value'],d['ms_per_step'])"
done; done
