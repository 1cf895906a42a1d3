# C2 exact fbank across library variants (LIBS), then PMC counters of the
# in-tree kernel.  Usage: LIBS="a.so b.so" bash tools/experiments/fb_variants.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/fbv
for k in 1 2; do
  for L in ${LIBS:-catears_amd/lib/libcatears_hip.so}; do
    v=$(basename $L .so)
    CATEARS_HIP_LIB=$R/$L timeout -k 10 120 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/fbv/$v.$k.json 2> gpurun_out/fbv/$v.$k.err || { tail -5 gpurun_out/fbv/$v.$k.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/fbv/$v.$k.json')); print('$v', round(l['value']/1e6,1), 'M frames/s', l['roofline']['frac'], l['checksum'])"
  done
done
[ -n "$PMC" ] && KREGEX=fbank_kernel WORKLOAD=c2 OUT=fbv/pmc bash tools/pmc_kernel.sh
exit 0
