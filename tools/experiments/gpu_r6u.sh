# C3 at the driver's flags over the nnet stream count around the default 8
# (20 steps: 8 streams take 3,3,3,3,2,2,2,2 batches, 7 take 3x6 + 2, 10 take
# 2 each), product library, A B C C B A x2 on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06u}
cd "$R" && mkdir -p gpurun_out/$T
for rep in 1 2; do
  for nb in 8 7 10 10 7 8; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --back-streams $nb \
        > gpurun_out/$T/c3_nb${nb}_$rep.json 2>gpurun_out/$T/c3_nb${nb}_$rep.err || { tail -5 gpurun_out/$T/c3_nb${nb}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_nb${nb}_$rep.json')); print('c3 streams $nb', round(l['value']/1e6, 4), 'M frames/s', l['ms_per_step'], l['roofline']['frac'], l['checksum'])"
  done
done
echo exit 0
