# Two-rank rehearsal of the driver's N=2 command on a one-GPU box: both ranks
# on device 0, gloo for the gather (RCCL needs distinct devices).  C3 and C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/n2
export CATEARS_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline > gpurun_out/n2/c3.json 2> gpurun_out/n2/c3.err || { tail -20 gpurun_out/n2/c3.err; exit 1; }
grep '^{' gpurun_out/n2/c3.json | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
    bench.py --workload c4 --gpus 2 --c4-utts 4000 --dist-backend gloo --no-cpu-baseline > gpurun_out/n2/c4.json 2> gpurun_out/n2/c4.err || { tail -20 gpurun_out/n2/c4.err; exit 1; }
grep '^{' gpurun_out/n2/c4.json | cut -c1-600
