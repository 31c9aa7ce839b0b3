"""The per-window exchange step of a sharded run, as the runner drives it over
torch.distributed (RCCL on GPUs, gloo in the CPU tests).

A context's exchange buffer holds one block of `xcap` records per peer; record 0 of a block is a
header whose `t` field is the number of records that follow (written on the device by the window's
token bucket, include/tgsim.h). Only those records travel: the counts are exchanged first (one
small all-to-all), then each block's used prefix goes point-to-point from its send-block view into
the peer's receive-block view (one batch of isend/irecv, ring order), where tgsim_advance_end reads it. Moving the full fixed-size
buffers instead would cost S x xcap x 32 B per rank per window regardless of the traffic."""
from __future__ import annotations

REC = 32  # bytes per tgsim_record


def exchange(send, recv, xcap: int, dist) -> int:
    """All-to-all of the used part of every peer block. send / recv: uint8 tensors of
    world * xcap * 32 bytes (device tensors for RCCL, CPU tensors for gloo). Returns the number of
    records received from other ranks. One host round trip (the counts); the blocks then travel as
    one batch of point-to-point transfers straight between the block views (no packing copies)."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    blk = xcap * REC
    cnt = send.view(torch.int64).view(world, xcap * 4)[:, 0].contiguous()
    cnt_in = torch.empty_like(cnt)
    dist.all_to_all_single(cnt_in, cnt)
    both = torch.stack([cnt, cnt_in]).cpu().tolist()
    out_n = [(1 + min(max(int(c), 0), xcap - 1)) * REC for c in both[0]]
    in_n = [(1 + min(max(int(c), 0), xcap - 1)) * REC for c in both[1]]
    ops = []
    for k in range(1, world):  # ring order: every rank sends to rank+k while receiving from rank-k
        dst, src = (rank + k) % world, (rank - k) % world
        ops.append(dist.P2POp(dist.isend, send[dst * blk:dst * blk + out_n[dst]], dst))
        ops.append(dist.P2POp(dist.irecv, recv[src * blk:src * blk + in_n[src]], src))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return sum(in_n[p] // REC - 1 for p in range(world) if p != rank)
