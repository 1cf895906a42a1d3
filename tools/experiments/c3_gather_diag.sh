# C3 two-rank gather vs one process per rank (run twice), per (rank, step)
# rows: which side differs when tests/test_gpu_c4.py::
# test_c3_two_ranks_gather_every_row fails.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/c3diag
export CATEARS_BENCH_DEVICE=0
A="--model tdnn-xs --steps 6 --warmup 2 --pool 8 --no-cpu-baseline"
for rep in $(seq ${REPS:-3}); do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + rep)) \
      bench.py $A --gpus 2 --dist-backend gloo --c3-dump /tmp/c3diag_two$rep.npz > gpurun_out/c3diag/two$rep.log 2>&1 || { tail -20 gpurun_out/c3diag/two$rep.log; exit 1; }
  for k in a b; do
    for r in 0 1; do
      timeout -k 10 200 python bench.py $A --fold-all --as-rank $r --c3-dump /tmp/c3diag_one$rep$k.$r.npz > gpurun_out/c3diag/one$rep$k.$r.log 2>&1 || { tail -20 gpurun_out/c3diag/one$rep$k.$r.log; exit 1; }
    done
  done
  python3 - $rep <<'PY'
import sys, numpy as np
rep = sys.argv[1]
def load(name):
    return dict(np.load(name))
two = load(f"/tmp/c3diag_two{rep}.npz")
one = {k: {} for k in "ab"}
for k in "ab":
    for r in (0, 1):
        one[k].update(load(f"/tmp/c3diag_one{rep}{k}.{r}.npz"))
def cmp(x, y):
    bad = []
    for key in sorted(x):
        if key not in y:
            bad.append((key, "missing")); continue
        d = np.nonzero(np.any(x[key].view(np.uint32) != y[key].view(np.uint32), axis=1))[0]
        if len(d):
            bad.append((key, len(d), int(d[0]), int(d[-1]), float(np.abs(x[key][d] - y[key][d]).max())))
    return bad or "none"
print("rep", rep, "one_a vs one_b:", cmp(one["a"], one["b"]), "| two vs one_a:", cmp(one["a"], two),
      "| two vs one_b:", cmp(one["b"], two), flush=True)
PY
done
rm -f /tmp/c3diag_*.npz
