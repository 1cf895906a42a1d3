# C3 at the driver's flags: how many of the last batches run on 128 x 128
# wide tiles while the pipeline drains (--wide-tiles last / ends / ends2 / last2),
# product library, A B C D D C B A x2 on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06t}
cd "$R" && mkdir -p gpurun_out/$T
for rep in 1 2; do
  for w in last ends ends2 last2 last2 ends2 ends last; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wide-tiles $w \
        > gpurun_out/$T/c3_${w}_$rep.json 2>gpurun_out/$T/c3_${w}_$rep.err || { tail -5 gpurun_out/$T/c3_${w}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_${w}_$rep.json')); print('c3 wide $w', round(l['value']/1e6, 4), 'M frames/s', l['ms_per_step'], l['roofline']['frac'], l['checksum'])"
  done
done
echo exit 0
