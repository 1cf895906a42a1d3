#!/bin/bash
# Latency A/B of two builds of the library: abtmp/old.so vs abtmp/new.so, alternating.
set -e
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in old new; do
  CATEARS_HIP_LIB=$PWD/abtmp/$v.so timeout -k 10 200 python tools/latency.py 300 > gpurun_out/lab_$v.txt 2>&1
  echo "$v $(grep 'latency    rows    70\|latency    rows   270' gpurun_out/lab_$v.txt | tr -s ' ' | tr '\n' ' ')"
done; done
