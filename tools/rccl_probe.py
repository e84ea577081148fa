"""Probe: can two RCCL ranks share one GPU on this pool?  Runs the collectives
comm.TorchComm issues on the nccl backend (all_reduce in place, all_gather,
all_to_all_single with uneven splits).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_probe.py
"""
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ['RANK'])
    world = int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    dev = torch.device('cuda', 0)
    x = torch.full((1000,), rank + 1, dtype=torch.int64, device=dev)
    dist.all_reduce(x)
    assert int(x[0]) == world * (world + 1) // 2, x[0]
    outs = [torch.empty(3, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, torch.full((3,), rank, dtype=torch.uint8, device=dev))
    assert [int(o[0]) for o in outs] == list(range(world))
    send_counts = [rank + 1 + r for r in range(world)]
    send = torch.cat([torch.full((c,), rank * 100 + r, dtype=torch.int64, device=dev)
                      for r, c in enumerate(send_counts)])
    rc = [r + 1 + rank for r in range(world)]
    out = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out, send, output_split_sizes=rc, input_split_sizes=send_counts)
    torch.cuda.synchronize()
    o = 0
    for r, c in enumerate(rc):
        assert bool((out[o:o + c] == r * 100 + rank).all()), (r, out[o:o + c])
        o += c
    dist.barrier()
    print('rccl probe rank %d ok' % rank, flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
