# One process per run, the C3 pipeline with every step's fbank output (raw),
# CMVN output (norm) and log-likelihoods dumped as the nnet stream saw them;
# runs compared pairwise to place a nondeterministic batch.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/c3diag
export CATEARS_DUMP_FEATS=1
A="--model tdnn-xs --steps 6 --warmup 2 --pool 8 --no-cpu-baseline --fold-all --as-rank 1 ${EXTRA}"
for k in $(seq ${RUNS:-6}); do
  timeout -k 10 200 python bench.py $A --c3-dump /tmp/c3f_$k.npz > gpurun_out/c3diag/f$k.log 2>&1 || { tail -20 gpurun_out/c3diag/f$k.log; exit 1; }
done
python3 - <<'PY'
import numpy as np, os
runs = [dict(np.load(f"/tmp/c3f_{k}.npz")) for k in range(1, int(os.environ.get("RUNS", 6)) + 1)]
ref = runs[0]
for n, x in enumerate(runs[1:], 2):
    bad = []
    for key in sorted(ref):
        d = np.nonzero(np.any(ref[key].view(np.uint32) != x[key].view(np.uint32), axis=1))[0]
        if len(d):
            bad.append((key, len(d), int(d[0]), int(d[-1])))
    print("run", n, "vs 1:", bad or "identical", flush=True)
PY
rm -f /tmp/c3f_*.npz
