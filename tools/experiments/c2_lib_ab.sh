#!/bin/bash
# C2 A/B of two builds of the library (abtmp/old.so vs abtmp/new.so), alternating.
set -e
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in old new; do
  CATEARS_HIP_LIB=$PWD/abtmp/$v.so timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline --steps 30 --warmup 3 > gpurun_out/c2ab_$v.out 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/c2ab_$v.out').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['checksum'])"
done; done
