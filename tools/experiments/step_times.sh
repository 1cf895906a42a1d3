#!/bin/bash
# When does each of the 20 timed C3 steps finish?  (bench.py --step-times),
# with and without the pre-warm.
set -e
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-profile --step-times"
for pw in 0 150 0 150; do
  timeout -k 10 240 $B --steps 20 --warmup 5 --prewarm-ms $pw > gpurun_out/st_pw$pw.out 2> gpurun_out/st_pw$pw.err
  tail -n 1 gpurun_out/st_pw$pw.err
  python -c "import json,sys;d=json.loads(open('gpurun_out/st_pw$pw.out').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['prewarm'])"
done
