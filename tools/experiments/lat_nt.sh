#!/bin/bash
# Latency mode: non-temporal partial (bit 0) / reduce output (bit 1) stores.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for nt in 0 1 2 3; do
  CATEARS_LAT_NT=$nt timeout -k 10 200 python tools/latency.py 300 > gpurun_out/lnt_$nt.txt 2>&1
  echo "nt=$nt $(grep 'latency    rows    70\|latency    rows   270' gpurun_out/lnt_$nt.txt | tr -s ' ' | tr '\n' ' ')"
done; done
