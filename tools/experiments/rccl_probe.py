"""Can two ranks share one GPU on the "nccl" (RCCL) backend?  Each rank sends
a seeded tensor to rank 0 with batch_isend_irecv (the RowGather pattern);
rank 0 checks the bytes.  Run as
  python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29561 tools/experiments/rccl_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    n, width = 4096, 3456
    if rank == 0:
        bufs = [torch.empty((n, width), device="cuda") for _ in range(1, world)]
        ops = [dist.P2POp(dist.irecv, b, p, None) for p, b in zip(range(1, world), bufs)]
    else:
        g = torch.Generator(device="cuda").manual_seed(rank)
        t = torch.randn((n, width), device="cuda", generator=g)
        ops = [dist.P2POp(dist.isend, t, 0, None)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    torch.cuda.synchronize()
    ok = True
    if rank == 0:
        for p, b in zip(range(1, world), bufs):
            g = torch.Generator(device="cuda").manual_seed(p)
            want = torch.randn((n, width), device="cuda", generator=g)
            ok &= bool(torch.equal(b, want))
        print(f"rccl probe: world {world} on one device, {n}x{width} fp32 per peer, bytes equal: {ok}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
